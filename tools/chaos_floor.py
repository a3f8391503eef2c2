#!/usr/bin/env python3
"""Chaos floor of the reference's LM scores (build container only; uses the oracle, which
reproduces the reference bit-for-bit on these inputs).

For every golden Bates set (PHCX / SUPERB, and the PFD sets' 22-score path), re-score each candidate with every scipy.optimize.leastsq start
point nudged by one ulp (numpy.nextafter toward +inf on the non-zero entries, SURVEY.md
Appendix B) and record, per score, the fraction of candidates whose value moves by more
than 1e-5 / 1e-3 relative.  A GPU result that disagrees with the reference no more often
than the reference disagrees with itself under a 1-ulp nudge is indistinguishable from it;
tests/test_bates22_gpu.py uses these floors as its class-C thresholds.
Writes tests/golden/chaos_floor.json.
"""
import json
import os
import sys
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle.bates as B  # noqa: E402
from golden_util import bates_inputs, load  # noqa: E402


def main():
    warnings.simplefilter("ignore")
    orig = B.leastsq

    def nudged(f, x0, args=(), **kw):
        x = np.array(x0, dtype=float).copy()
        nz = x != 0
        x[nz] = np.nextafter(x[nz], np.inf)
        return orig(f, x, args=args, **kw)

    res = {}
    for name in ("bates22_phcx128", "bates22_superb64"):
        d = load(name)
        prof, sub, curve, scal = bates_inputs(d)
        B.leastsq = orig
        a, sa = B.bates22(prof, sub, curve, scal)
        B.leastsq = nudged
        b, sb = B.bates22(prof, sub, curve, scal)
        B.leastsq = orig
        ok = ((sa & 0xFF) == 0) & ((sb & 0xFF) == 0)
        with np.errstate(all="ignore"):
            r = np.abs(a - b) / np.maximum(np.abs(a), 1e-300)
        r[(a == b) | (np.isnan(a) & np.isnan(b))] = 0.0
        r[np.isnan(r)] = np.inf
        r = r[ok]
        res[name] = {"n": int(ok.sum()),
                     "moved_1e-5": np.round((r > 1e-5).mean(axis=0), 4).tolist(),
                     "moved_1e-3": np.round((r > 1e-3).mean(axis=0), 4).tolist()}
        print(name, res[name], flush=True)
    # the PFD 22-score sets (oracle/pfd.bates22_one on the folds rebuilt from the seeds)
    import tempfile

    from oracle import pfd as opfd
    from pulsarfeatureextractor_amd import pfd as P
    from test_oracle_pfd import SETS, build_files, load_set

    def pfd_rows(datas):
        out = np.full((len(datas), 22), np.nan)
        ok = np.zeros(len(datas), dtype=bool)
        for i, dd in enumerate(datas):
            try:
                out[i] = opfd.bates22_one(dd)[0]
                ok[i] = True
            except B.CandidateFailure:
                pass
        return out, ok

    for name in SETS:
        g = load_set(name)
        with tempfile.TemporaryDirectory() as tmp:
            datas = [P.read(f) for f in build_files(tmp, g)]
        B.leastsq = orig
        a, oka = pfd_rows(datas)
        B.leastsq = nudged
        b, okb = pfd_rows(datas)
        B.leastsq = orig
        ok = oka & okb
        with np.errstate(all="ignore"):
            r = np.abs(a - b) / np.maximum(np.abs(a), 1e-300)
        r[(a == b) | (np.isnan(a) & np.isnan(b))] = 0.0
        r[np.isnan(r)] = np.inf
        r = r[ok]
        res[name] = {"n": int(ok.sum()),
                     "moved_1e-5": np.round((r > 1e-5).mean(axis=0), 4).tolist(),
                     "moved_1e-3": np.round((r > 1e-3).mean(axis=0), 4).tolist()}
        print(name, res[name], flush=True)
    with open(os.path.join(ROOT, "tests", "golden", "chaos_floor.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
