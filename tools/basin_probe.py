#!/usr/bin/env python3
"""Which minima does the reference's own T1 fit reach under ulp-level path noise?

fitGaussianT1 -> fitGaussianWithBackground (ProfileOperations.py:1061-1264) is re-run by the
oracle (scipy.optimize.leastsq, as the reference) on one synthetic candidate with every
residual evaluation multiplied by (1 + u 2^-k), u ~ U(-1, 1) drawn afresh per evaluation --
the kind of last-bit differences a different summation order produces at every LM step.
The distinct chi^2 values (s9) reached over 24 seeds are printed with their counts.  Used in
DESIGN.md §4 for the lp=200 candidate where the GPU's s9 (1755.368) differs from the
oracle's noiseless path (1693.103): the reference reaches 1755.368 itself under such noise.

  python tools/basin_probe.py [lp n seed row]        (defaults: 200 48 1200 31)
"""
import os
import sys
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle.bates as B  # noqa: E402
from pulsarfeatureextractor_amd.synth import bates_batch  # noqa: E402


def main(lp=200, n=48, seed=1200, row=31):
    warnings.simplefilter("ignore")
    b = bates_batch(n, lp=lp, lsb=lp, seed=seed)
    p = b["prof"][row].astype(np.int64)
    hp = B.histogram(p, B.fd_bins(p))
    _s, p_mu, _a = B.fit_gaussian_hist(hp[1], hp[0])[0]
    minbg = min(p_mu, p.mean())
    tp = [max(v - minbg + p.std(), 0.0) for v in p] if minbg > 0 else p
    y, _cut = B._rotate_half(tp)
    y = np.asarray(y, dtype=float)
    x = np.arange(len(y))
    e = int(np.argmax(y))
    print(f"candidate {row} of bates_batch({n}, lp={lp}, seed={seed}): T1 fit, s9 reached")
    for k in (53, 50, 45):
        outs = []
        for s in range(24):
            rng = np.random.default_rng(s)

            def f(p_, x_, y_):
                r = y_ - B._gbg(x_, p_)
                return r * (1 + rng.uniform(-1, 1, r.shape) * 2.0 ** -k)

            pp = B.leastsq(f, [np.std(y), e, y[e], 1.0], args=(x, y))[0]
            fit = B._gbg(x, pp)
            outs.append(round(float(np.sum((y - fit) ** 2) / len(y)), 3))
        vals = sorted(set(outs))
        print(f"  noise 2^-{k}: " + ", ".join(f"{v} x{outs.count(v)}" for v in vals))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:5]])
