#!/usr/bin/env python3
"""Run-to-run determinism of pfe_bates22 on one input set: score the set R times (plus R
times with the groups serialised and R times with the hand-over off) and report every row /
score whose bits differ from the first run.
  python tools/determinism_probe.py [--set bates22_phcx128] [--reps 12] [--tile 1]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="bates22_phcx128")
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--tile", type=int, default=1, help="repeat the set this many times per call")
    a = ap.parse_args()
    from golden_util import bates_inputs, load
    from pulsarfeatureextractor_amd._native import Engine

    prof, sub, curve, scal = bates_inputs(load(a.set))
    n = len(prof)
    t = a.tile
    prof, sub, curve, scal = (np.concatenate([x] * t) for x in (prof, sub, curve, scal))
    res = {}
    with Engine(0) as e:
        for tag, opts in (("default", {}), ("serial", {"serial": 1}), ("nohand", {"handover": 0})):
            runs = []
            for _ in range(a.reps):
                with e.options(**opts):
                    o, s = e.bates22(prof, sub, curve, scal)
                runs.append(np.nan_to_num(o, nan=7.0).view(np.int64).copy())
            ref = runs[0]
            diff = {}
            for r in runs[1:]:
                rows, cols = np.nonzero(r != ref)
                for i, j in zip(rows.tolist(), cols.tolist()):
                    diff.setdefault(f"s{j + 1}", set()).add(i % n)
            # tiles of one call must agree too (a candidate's scores must not depend on its slot)
            tiles = ref.reshape(t, n, 22)
            trow, tcol = np.nonzero((tiles != tiles[:1]).any(axis=0))
            res[tag] = {"runs_differing_rows": {k: sorted(v) for k, v in diff.items()},
                        "tile_differing": sorted(set(trow.tolist())), "tile_cols": sorted(set(tcol.tolist()))}
            print(tag, json.dumps(res[tag]), flush=True)


if __name__ == "__main__":
    main()
