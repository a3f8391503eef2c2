#!/usr/bin/env python3
"""Per-candidate stability of the reference's LM scores (build container only; test data).

tools/chaos_floor.py measures, per score, the FRACTION of candidates whose value moves
when every scipy.optimize.leastsq start point is nudged by one ulp.  This tool records
WHICH candidates move: each golden Bates set is re-scored by the oracle (bit-exact to the
reference on these inputs, tests/test_oracle_golden.py) under several perturbations of
the start points -- +-1, +-2 and +4 ulp of every non-zero entry (SURVEY.md
Appendix B: zero entries stay zero) -- and of the residuals (two fixed patterns of
+-1 ulp on the residual vector the solver sees), and the largest relative change of every
score over the perturbations is stored per candidate:

    tests/golden/chaos_rows.npz   <set>_rmax  (n, 22) float64
                                  (inf where a perturbation changes whether the candidate
                                   fails, 0 for candidates the reference fails)

tests/test_bates22_gpu.py holds the GPU to 1e-5 on every (candidate, score) whose rmax is
<= STABLE (the reference's own answer is stable there), and to the population floor only
on the rest.
"""
import os
import sys
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle.bates as B  # noqa: E402
from golden_util import bates_inputs, load  # noqa: E402

SETS = ("bates22_phcx128", "bates22_superb64", "all30_phcx128", "bates22_phcx128_wide")


def nudger(orig, steps):
    def nudged(f, x0, args=(), **kw):
        x = np.array(x0, dtype=float).copy()
        nz = x != 0
        for _ in range(abs(steps)):
            x[nz] = np.nextafter(x[nz], np.inf if steps > 0 else -np.inf)
        return orig(f, x, args=args, **kw)

    return nudged


def residual_noise(orig, seed):
    """Every residual vector the solver evaluates multiplied element-wise by 1 + u_i 2^-53,
    u_i in {-1, 0, 1} from a fixed pattern: last-bit differences in the function values, the
    kind a different evaluation or summation order produces."""
    def nudged(f, x0, args=(), **kw):
        def g(x, *a):
            r = np.asarray(f(x, *a), dtype=float)
            u = np.random.default_rng(seed + r.size).integers(-1, 2, size=r.shape)
            return r * (1.0 + u * 2.0 ** -53)
        return orig(g, x0, args=args, **kw)

    return nudged


def rel(a, b):
    with np.errstate(all="ignore"):
        r = np.abs(a - b) / np.maximum(np.abs(a), 1e-300)
    r[(a == b) | (np.isnan(a) & np.isnan(b))] = 0.0
    r[np.isnan(r)] = np.inf
    return r


def main():
    warnings.simplefilter("ignore")
    orig = B.leastsq
    res = {}
    for name in SETS:
        d = load(name)
        prof, sub, curve, scal = bates_inputs(d)
        a, sa = B.bates22(prof, sub, curve, scal)
        oka = (sa & 0xFF) == 0
        rmax = np.zeros_like(a)
        try:
            for pert in (1, -1, 2, -2, 4, "r1", "r2"):
                B.leastsq = (nudger(orig, pert) if isinstance(pert, int)
                             else residual_noise(orig, 7 if pert == "r1" else 11))
                b, sb = B.bates22(prof, sub, curve, scal)
                okb = (sb & 0xFF) == 0
                r = rel(a, b)
                r[oka != okb] = np.inf
                r[~oka & ~okb] = 0.0
                rmax = np.maximum(rmax, r)
        finally:
            B.leastsq = orig
        res[f"{name}_rmax"] = rmax
        stable = (rmax <= 1e-7)[oka]
        print(name, "stable fraction per score:", np.round(stable.mean(axis=0), 3).tolist(), flush=True)
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "chaos_rows.npz"), **res)


if __name__ == "__main__":
    main()
