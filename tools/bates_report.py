#!/usr/bin/env python3
"""Per-score agreement report: pfe_bates22 (GPU) vs the reference's golden vectors.

Prints, for each of the 22 scores, the fraction of candidates agreeing bitwise, within
1e-9, 1e-5 and 1e-3 relative, plus the failure-pattern agreement.  Used to set and justify
the parity thresholds in tests/test_bates22_gpu.py.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from golden_util import bates_inputs, load  # noqa: E402
from pulsarfeatureextractor_amd._native import Engine  # noqa: E402


def agreement(got, ref):
    with np.errstate(all="ignore"):
        same = (got == ref) | (np.isnan(got) & np.isnan(ref))
        rel = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-300)
        rel[same] = 0.0
        rel[np.isnan(rel)] = np.inf
    return {
        "bitwise": same.mean(axis=0).round(4).tolist(),
        "1e-9": (rel <= 1e-9).mean(axis=0).round(4).tolist(),
        "1e-5": (rel <= 1e-5).mean(axis=0).round(4).tolist(),
        "1e-3": (rel <= 1e-3).mean(axis=0).round(4).tolist(),
    }


def main():
    rep = {}
    saved = {}
    with Engine(0) as e:
        for name in ("bates22_phcx128", "bates22_superb64", "all30_phcx128"):
            d = load(name)
            prof, sub, curve, scal = bates_inputs(d)
            t0 = time.time()
            out, st = e.bates22(prof, sub, curve, scal)
            dt = time.time() - t0
            ok = d["ok"]
            gok = (st & 0xFF) == 0
            m = ok & gok
            ref = d["out"][:, -22:]  # all30: the 22 scores follow the 8 Lyon features
            r = agreement(out[m], ref[m])
            r["fail_pattern_equal"] = bool(np.array_equal(ok, gok))
            r["ref_fail"] = np.where(~ok)[0].tolist()
            r["gpu_fail"] = np.where(~gok)[0].tolist()
            r["gpu_status"] = [int(x) for x in st[~gok]]
            r["seconds"] = dt
            rep[name] = r
            saved[name + "_out"] = out
            saved[name + "_st"] = st
            # the same candidates through the batched solver: agreement between two GPU solvers
            # that differ only in the order of their m-sums (same sin/exp code)
            with e.options(solver="batched"):
                ob, sb = e.bates22(prof, sub, curve, scal)
            saved[name + "_batched"] = ob
            mb = m & ((sb & 0xFF) == 0)
            r2 = agreement(ob[mb], out[mb])
            print(name, "pooled vs batched", json.dumps(r2), flush=True)
            rep[name + "_pooled_vs_batched"] = r2
    if "--save" in sys.argv:
        np.savez_compressed(sys.argv[sys.argv.index("--save") + 1], **saved)
    return rep


if __name__ == "__main__":
    main()
