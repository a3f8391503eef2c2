#!/usr/bin/env python3
"""Determinism probe: the all30 golden set's 22 scores, several times in one process (fresh
handle and reused handle), printed for the rows given (default: 5)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from golden_util import bates_inputs, load  # noqa: E402
from pulsarfeatureextractor_amd._native import Engine  # noqa: E402

rows = [int(v) for v in sys.argv[1:]] or [5]
d = load("all30_phcx128")
prof, sub, curve, scal = bates_inputs(d)
outs = []
for h in range(2):
    with Engine(0) as e:
        for k in range(3):
            o, s = e.bates22(prof, sub, curve, scal)
            outs.append(o)
            print(f"handle {h} call {k}: " + " ".join(f"r{r}: s8 {o[r, 7]!r} s9 {o[r, 8]!r}" for r in rows))
        o8 = e.lyon8(prof, d["block0"])
        o, s = e.bates22(prof, sub, curve, scal)
        print(f"handle {h} after lyon8: " + " ".join(f"r{r}: s8 {o[r, 7]!r} s9 {o[r, 8]!r}" for r in rows))
        outs.append(o)
ref = np.nan_to_num(outs[0], nan=7.0)
for i, o in enumerate(outs):
    diff = np.argwhere(np.nan_to_num(o, nan=7.0) != ref)
    print(f"run {i}: {len(diff)} differing cells vs run 0", diff[:8].tolist())
print("gold", [(d["out"][r, 15], d["out"][r, 16]) for r in rows])
