"""Load tests/golden/*.npz (made by tools/make_golden.py from the reference itself)."""
import os

import numpy as np

from pulsarfeatureextractor_amd.phcx import reduce_dm_curve

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# score classes; 0-based columns
CLASS_C = (6, 7, 8, 9, 10, 16, 17)        # s7-s11, s17, s18: ill-conditioned LM outputs
CLASS_E = (2,)                            # s3: integer peak count
SELF_NOISY = (9, 10)                      # s10, s11: the reference disagrees with itself


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def bates_inputs(d):
    """Arrays in the libpfe layout from a bates22 golden set."""
    superb = bool(d["superb"])
    blk = d["block0"] if superb else d["block1"]
    curves = np.stack([reduce_dm_curve(b)[0] for b in blk])
    n = len(d["ok"])
    scal = np.zeros((n, 8))
    scal[:, 0] = d["period"] * 1000
    scal[:, 1] = d["snr"]
    scal[:, 2] = d["dm"]
    scal[:, 3] = d["width"]
    scal[:, 4] = d["dm_start"]
    scal[:, 5] = d["dm_end"]
    scal[:, 6] = blk.shape[1]
    return d["prof"], d["sub"], curves, scal


def oracle_with_floor(prof, sub, curve, scal):
    """Oracle scores of a fresh batch plus that batch's own chaos floor: the fraction of
    candidates whose score moves (> 1e-5 / > 1e-3 relative) when every leastsq start point
    is nudged by one ulp (the tools/chaos_floor.py procedure, applied to this batch)."""
    import warnings

    import oracle.bates as B

    orig = B.leastsq

    def nudged(f, x0, args=(), **kw):
        x = np.array(x0, dtype=float).copy()
        nz = x != 0
        x[nz] = np.nextafter(x[nz], np.inf)
        return orig(f, x, args=args, **kw)

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a, sa = B.bates22(prof, sub, curve, scal)
        try:
            B.leastsq = nudged
            b, sb = B.bates22(prof, sub, curve, scal)
        finally:
            B.leastsq = orig
    ok = ((sa & 0xFF) == 0) & ((sb & 0xFF) == 0)
    with np.errstate(all="ignore"):
        r = np.abs(a - b) / np.maximum(np.abs(a), 1e-300)
    r[(a == b) | (np.isnan(a) & np.isnan(b))] = 0.0
    r[np.isnan(r)] = np.inf
    r = r[ok]
    floor = {"moved_1e-5": (r > 1e-5).mean(axis=0).tolist(),
             "moved_1e-3": (r > 1e-3).mean(axis=0).tolist()}
    return a, sa, floor
