#!/usr/bin/env python3
"""Algorithmic fp64 operation count of the 22-score path per candidate.

Counts the work MINPACK lmdif does on each solve, not the instructions a GPU issues: the
solve statistics (solves, Jacobians, lmpar/qrsolv calls and function evaluations per solve,
per parameter count) come from the instrumented build (tools/lm_profile.py JSON); the model
cost per residual element and the residual count m per solve group are stated below.  Every
add/sub/mul/div/sqrt/exp/sin counts as one operation.

  python tools/bates_flops.py gpurun_out/lmprof.json > profiles/r01_bates22_flops.json
"""
import json
import sys

import numpy as np


def qrfac_ops(m, n):
    """Householder QR with column pivoting (MINPACK qrfac), m x n."""
    ops = 2 * m * n  # initial column norms
    for j in range(n):
        mj = m - j
        ops += 2 * mj + 1 + mj + 1  # column norm, sign, scale, +1
        for _c in range(j + 1, n):
            ops += 2 * mj + 1 + 2 * mj + 6  # dot, /ajj, axpy, rdiag downdate
    return ops


def qtf_ops(m, n):
    return sum(4 * (m - j) + 2 for j in range(n))


def qrsolv_ops(n):
    rot = n * (n + 1) // 2
    return rot * 12 + sum(6 * (n - k - 1) for j in range(n) for k in range(j, n)) + n * n + 2 * n


def lmpar_ops(n):
    return 6 * n * n + 30 * n


# model cost per residual element and residual count per solve group (lp = ndm = 128)
GROUPS = {
    # key in lm_profile JSON: (ops per residual element, m, what)
    "gauss/N=2": (8, None, "fitGaussianFixedWidthBins on the profile histogram (m = bins)"),
    "gauss/N=3": (8, None, "fitGaussian on the dy and profile histograms, with retries (m = bins)"),
    "gauss/N=4": (9, 128, "fitGaussianWithBackground (T1) + 8 peel passes of fitDoubleGaussian"),
    "gauss/N=8": (18, 128, "fitDoubleGaussianWithBackground"),
    "sine_dm_sub/N=2": (7.5, 128, "fitSine + fitSineSqr"),
    "sine_dm_sub/N=3": (15, 128, "DM-curve fit"),
}


def mean_hist_bins(n=2000, lp=128):
    sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
    from oracle.bates import backward_diff, fd_bins
    from pulsarfeatureextractor_amd.synth import bates_batch

    b = bates_batch(n, lp=lp, seed=31)
    hp = [fd_bins(p.astype(np.float64)) for p in b["prof"]]
    hd = [fd_bins(backward_diff(p.astype(np.float64))) for p in b["prof"]]
    return float(np.mean(hp)), float(np.mean(hd))


def main():
    prof = json.load(open(sys.argv[1]))
    hp, hd = mean_hist_bins()
    n_cand = prof["gauss/N=8"]["calls"]
    total = 0.0
    groups = {}
    for key, (c_model, m, what) in GROUPS.items():
        g = prof[key]
        if m is None:
            m = hp if key == "gauss/N=2" else 0.5 * (hp + hd)
        npar = int(key.split("N=")[1])
        calls = g["calls"] / n_cand
        iters = g["iters_per_call"]
        lmpar = g["lmpar_per_iter"] * iters
        qrs = g["qrsolv_per_lmpar"] * lmpar
        nfev = g["nfev_per_call"]
        per_solve = (nfev * m * c_model + iters * (npar * m * 2 + qrfac_ops(m, npar) + qtf_ops(m, npar)
                     + 2 * npar * npar) + lmpar * (lmpar_ops(npar) + 2 * m + 20) + qrs * qrsolv_ops(npar))
        groups[key] = {"what": what, "solves_per_candidate": calls, "m": m, "n": npar,
                       "nfev_per_solve": nfev, "jacobians_per_solve": iters,
                       "ops_per_solve": per_solve, "ops_per_candidate": per_solve * calls}
        total += per_solve * calls
    # non-LM work: histograms, percentiles, boxcars, 120 sub-band correlations, chi^2 sums
    other = 16 * 128 * 3 + 120 * 128 * 6 + 17 * 128 * 6 + 20 * 128
    print(json.dumps({"ops_per_candidate": total + other, "lm_ops_per_candidate": total,
                      "other_ops_per_candidate": other, "mean_hist_bins_profile": hp,
                      "mean_hist_bins_dy": hd, "groups": groups,
                      "source": sys.argv[1]}, indent=1))


if __name__ == "__main__":
    main()
