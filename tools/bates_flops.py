#!/usr/bin/env python3
"""Algorithmic fp64 operation count of the 22-score path per candidate.

Counts the work MINPACK lmdif does on each solve, not the instructions a GPU issues: the
solve statistics (solves, Jacobians, lmpar/qrsolv calls and function evaluations per solve,
per parameter count) come from the instrumented build (tools/lm_profile.py JSON); the model
cost per residual element and the residual count m per solve group are stated below.  Every
add/sub/mul/div/sqrt/exp/sin counts as one operation.

  python tools/bates_flops.py gpurun_out/lmprof.json > profiles/r01_bates22_flops.json
  python tools/bates_flops.py --pfd gpurun_out/r03_lmprof_pfd22.json > profiles/r03_pfd22_ops.json

--pfd: the PFD 22-score path (PFDFile.compute, PFDFile.py:587-613) on bench.py's 16 x 32 x 128
folds: the same Gaussian / sine fits on the float 0..255 profile (histogram widths measured on
that profile), the PFD DM-curve fit (PFDOperations.getDMFittings :274-393: N = 4, m = 100
trial DMs, 14 operations per residual), and the fold arithmetic of pfe_pfd_dmprof (part sums,
the 100-DM chi^2 sweep) plus the sub-band correlations as non-LM work.
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


PFD_SHAPE = (16, 32, 128)  # npart x nsub x proflen of bench.py --path pfd22
PFD_NDM = 100              # PFDFile.plot_chi2_vs_DM trial DMs


def pfd_groups():
    g = {k: v for k, v in GROUPS.items() if not k.startswith("sine_dm_sub/N=3")}
    g["pfd22/N=4"] = (14, PFD_NDM, "PFD DM-curve fit (getDMFittings, m = 100 trial DMs)")
    return g


def mean_hist_bins_pfd(n=300):
    """FD widths of the PFD profile (pfe_pfd_dmprof's 0..255 float profile) and its
    derivative, over bench.py's synthetic folds."""
    root = __file__.rsplit("/tools/", 1)[0]
    sys.path.insert(0, root)
    from bench import pfd_block
    from oracle.bates import backward_diff, fd_bins
    from oracle.pfd import PFDState

    hp, hd = [], []
    for d in pfd_block(n, PFD_SHAPE, 20261019):
        p = np.asarray(PFDState(d).profile(), dtype=np.float64)
        hp.append(fd_bins(p))
        hd.append(fd_bins(backward_diff(p)))
    return float(np.mean(hp)), float(np.mean(hd))


def pfd_other_ops():
    npart, nsub, L = PFD_SHAPE
    parts = npart * nsub * L            # part sums (dedisperse at the best DM)
    sweep = PFD_NDM * (nsub * L + 3 * L)  # per trial DM: rotated sub-band sums + chi^2
    sub = 120 * L * 6 + 17 * L * 6 + 20 * L  # sub-band correlations, boxcars
    return parts + sweep + sub + 16 * L * 3


def main():
    pfd = "--pfd" in sys.argv
    src = [a for a in sys.argv[1:] if not a.startswith("--")][0]
    prof = json.load(open(src))
    # the Gaussian chain is three translation units, each with its own counter set
    for k in list(prof):
        if k.startswith(("gauss_peel/", "gauss_dg8/")):
            prof.setdefault("gauss/" + k.split("/", 1)[1], prof[k])
    hp, hd = mean_hist_bins_pfd() if pfd else mean_hist_bins()
    n_cand = prof["gauss/N=8"]["calls"]
    total = 0.0
    groups = {}
    for key, (c_model, m, what) in (pfd_groups() if pfd else GROUPS).items():
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
    other = pfd_other_ops() if pfd else 16 * 128 * 3 + 120 * 128 * 6 + 17 * 128 * 6 + 20 * 128
    print(json.dumps({"ops_per_candidate": total + other, "lm_ops_per_candidate": total,
                      "other_ops_per_candidate": other, "mean_hist_bins_profile": hp,
                      "mean_hist_bins_dy": hd, "groups": groups,
                      "source": src, "path": "pfd22" if pfd else "bates22"}, indent=1))


if __name__ == "__main__":
    main()
