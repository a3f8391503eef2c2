#!/usr/bin/env python3
"""Row-conditioned parity report of the 22 scores (host only, from a GPU dump).

Input: the npz tools/bates_report.py --save writes on the GPU box (GPU scores of the golden
sets with the pooled and the batched solver) and tests/golden/chaos_rows.npz.  For every
score it prints:
  stable    fraction of candidates whose reference score moves by <= 1e-7 under all seven
            perturbations of tools/chaos_rows.py
  bad@st    candidates among those where the GPU differs from the reference by > 1e-5
  1e-5      fraction of all candidates where the GPU is within 1e-5 of the reference
  bitwise   fraction bit-identical to the reference
  pb-bit    fraction where the pooled and the batched GPU solvers agree bit for bit (same
            sin/exp code, only the order of the m-sums differs)

  python tools/parity_report.py gpurun_out/r02_golden_gpu.npz > profiles/r02_parity_rows.txt
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from golden_util import load  # noqa: E402

STABLE = 1e-7


def rel(a, b):
    with np.errstate(all="ignore"):
        r = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    r[(a == b) | (np.isnan(a) & np.isnan(b))] = 0.0
    r[np.isnan(r)] = np.inf
    return r


def main(path):
    g = np.load(path)
    rows = np.load(os.path.join(ROOT, "tests", "golden", "chaos_rows.npz"))
    for name in ("bates22_phcx128", "bates22_superb64", "all30_phcx128"):
        d = load(name)
        ref = d["out"][:, -22:]
        ok = d["ok"] & ((g[name + "_st"] & 0xFF) == 0)
        out, ob = g[name + "_out"][ok], g[name + "_batched"][ok]
        r = rel(out, ref[ok])
        rpb = rel(ob, out)
        stable = rows[name + "_rmax"][ok] <= STABLE
        print(f"{name}: {ok.sum()} scored candidates (stable: reference moves <= {STABLE:g} "
              f"under the 7 perturbations)")
        print(f"{'score':>6} {'stable':>7} {'bad@st':>7} {'1e-5':>7} {'bitwise':>8} {'pb-bit':>7}")
        for j in range(22):
            bad = int((stable[:, j] & (r[:, j] > 1e-5)).sum())
            print(f"{'s' + str(j + 1):>6} {stable[:, j].mean():7.3f} {bad:7d} "
                  f"{(r[:, j] <= 1e-5).mean():7.3f} {(r[:, j] == 0).mean():8.3f} "
                  f"{(rpb[:, j] == 0).mean():7.3f}")
        print()


if __name__ == "__main__":
    main(sys.argv[1])
