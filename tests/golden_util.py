"""Load tests/golden/*.npz (made by tools/make_golden.py from the reference itself)."""
import os
import sys

import numpy as np

from pulsarfeatureextractor_amd.phcx import reduce_dm_curve

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# score classes; 0-based columns
CLASS_C = (6, 7, 8, 9, 10, 16, 17)        # s7-s11, s17, s18: ill-conditioned LM outputs
CLASS_E = (2,)                            # s3: integer peak count
SELF_NOISY = (9, 10)                      # s10, s11: the reference disagrees with itself


ENVELOPE_TOL = 1e-5   # the north star's relative bar, applied at both ends of an envelope
ENVELOPE_TIGHT = 1e-7  # an envelope narrower than this (relative) is a reproducible value
# scores that are outputs of ONE least-squares fit (0-based columns): s8/s9 (fitGaussianT1),
# s10/s11 (the double-Gaussian fit), s17/s18 (the DM-curve fit).  A fit is reproducible on a
# row only if all of its outputs are: when the reference's samples spread on one of them the
# fit changes basin on that row, and its other outputs are one more draw of the same process
FIT_GROUPS = ((7, 8), (9, 10), (16, 17))


def envelope_check(out, st, name, skip=(), cols=slice(None)):
    """Row-by-row pin of a golden set's LM scores against the reference's own spread
    (tests/golden/chaos_envelope.npz, tools/chaos_envelope.py: per candidate the min / max
    over K = 50 samples -- the golden value, the oracle's own run and 48 ulp-scale nudges of
    start points and residuals).

      * tight rows (the K samples agree to 1e-7 on this score and on every other output of
        the same fit, FIT_GROUPS): the GPU value must lie inside
        [lo - 1e-5 |lo|, hi + 1e-5 |hi|] -- every such row, s10/s11 included;
      * wide rows (the reference itself spreads): the GPU value is one more draw of the same
        chaotic process and falls outside the K samples' range with probability p = 2/(K+1);
        the count outside is held to n p + 3 sqrt(n p (1-p)) + 1.

    Rows the reference fails, or whose failure status changes under a nudge, are skipped
    (the failure pattern itself is checked exactly by the callers).  Returns per-score
    statistics {score: (tight rows, wide rows, outside wide, bound)}."""
    env = np.load(os.path.join(GOLDEN, "chaos_envelope.npz"))
    d = load(name)
    lo, hi, fixed = env[f"{name}_lo"], env[f"{name}_hi"], env[f"{name}_fixed"]
    gold = d["out"][:, cols]
    k = len(env["runs"]) + 1
    p = 2.0 / (k + 1)
    ok = d["ok"].astype(bool) & fixed & ((st & 0xFF) == 0)
    with np.errstate(all="ignore"):
        inside = (out >= lo - ENVELOPE_TOL * np.abs(lo)) & (out <= hi + ENVELOPE_TOL * np.abs(hi))
        tight = (hi - lo) <= ENVELOPE_TIGHT * np.maximum(np.abs(lo), np.abs(hi))
    for grp in FIT_GROUPS:
        cols_g = [j for j in grp if j < tight.shape[1]]
        both = np.logical_and.reduce([tight[:, j] for j in cols_g])
        for j in cols_g:
            tight[:, j] = both
    inside |= (out == gold) | (np.isnan(out) & np.isnan(gold))
    stats = {}
    for j in range(22):
        if j in skip:
            continue
        t, w = ok & tight[:, j], ok & ~tight[:, j]
        bad_t = np.where(t & ~inside[:, j])[0]
        assert len(bad_t) == 0, (f"{name}: s{j + 1} outside the reference's envelope on "
                                 f"{len(bad_t)} rows where it is tight (rows {bad_t[:10].tolist()})")
        nw = int(w.sum())
        out_w = int((w & ~inside[:, j]).sum())
        bound = nw * p + 3.0 * np.sqrt(nw * p * (1 - p)) + 1.0
        assert out_w <= bound, (f"{name}: s{j + 1} outside the reference's envelope on {out_w} "
                                f"of {nw} chaotic rows (binomial bound {bound:.1f} at p = {p:.3f})")
        stats[j + 1] = (int(t.sum()), nw, out_w, bound)
    return stats


class _Set(dict):
    """A golden set assembled in memory (same keys as the .npz sets)."""

    @property
    def files(self):
        return list(self.keys())


def _label_phcx_set():
    """The PHCX candidates of the --label golden (tests/golden/label.npz) as a bates22 set:
    inputs phcx_in_*, 'out' = the 22 scores the reference wrote to Scores.csv (Python 3
    repr, so the golden values are exact), 'ok' = listed in Cands.meta."""
    g = np.load(os.path.join(GOLDEN, "label.npz"))
    d = _Set({k[len("phcx_in_"):]: g[k] for k in g.files if k.startswith("phcx_in_")})
    n = int(d["n"])
    out = np.full((n, 22), np.nan)
    ok = np.zeros(n, dtype=bool)
    for ln in str(g["phcx_Scores.csv"]).splitlines():
        if not ln:
            continue
        vals, name = ln.rsplit(",%", 1)
        i = int(name.rsplit("label_", 1)[1].split(".")[0])
        out[i] = [float(v) for v in vals.split(",")[:-1]]
        ok[i] = True
    d.update(out=out, ok=ok, superb=np.bool_(False))
    return d


def load(name):
    if name == "label_phcx":
        return _label_phcx_set()
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def bates_inputs(d):
    """Arrays in the libpfe layout from a bates22 golden set."""
    superb = bool(d["superb"])
    if "dmcurve" in d:  # compact sets store the reduced curves and the block length
        curves, blen = d["dmcurve"], int(d["block_len"])
    else:
        blk = d["block0"] if superb else d["block1"]
        curves = np.stack([reduce_dm_curve(b)[0] for b in blk])
        blen = blk.shape[1]
    n = len(d["ok"])
    scal = np.zeros((n, 8))
    scal[:, 0] = d["period"] * 1000
    scal[:, 1] = d["snr"]
    scal[:, 2] = d["dm"]
    scal[:, 3] = d["width"]
    scal[:, 4] = d["dm_start"]
    scal[:, 5] = d["dm_end"]
    scal[:, 6] = blen
    return d["prof"], d["sub"], curves, scal


# the unperturbed pass, the seven nudges, and the unperturbed pass once more: numpy's SIMD
# reductions follow the heap alignment of their operands, so a second run (later in the
# process, or in another spawned one) is a sample of the reference's own spread too (a row
# whose fit changes basin between the two is not "stable")
_PERTS = (None, 1, -1, 2, -2, 4, "r7", "r11", None)


def _oracle_run(args):
    """One oracle pass over a batch under perturbation `pert` (None: unperturbed)."""
    pert, prof, sub, curve, scal = args
    import warnings

    import oracle.bates as B

    tools = os.path.join(os.path.dirname(GOLDEN), "..", "tools")
    if tools not in sys.path:
        sys.path.insert(0, tools)
    from chaos_rows import nudger, residual_noise

    orig = B.leastsq
    if pert is not None:
        B.leastsq = nudger(orig, pert) if isinstance(pert, int) else residual_noise(orig, int(pert[1:]))
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            return B.bates22(prof, sub, curve, scal)
    finally:
        B.leastsq = orig


def oracle_with_floor(prof, sub, curve, scal, workers=1):
    """Oracle scores of a fresh batch plus that batch's own chaos data (tools/chaos_rows.py,
    applied to this batch): every leastsq start point nudged by +-1, +-2 and +4 ulp, two
    patterns of +-1 ulp on the residuals, and a second unperturbed pass in another heap state.  Returns (scores, status, floor, rmax): floor = the
    fraction of candidates whose score moves by > 1e-5 / > 1e-3 relative under any of them,
    rmax (n, 22) = each candidate's largest relative move.  workers > 1: the nine passes run
    in spawned processes (no state is copied from a parent that holds a GPU context)."""
    tools = os.path.join(os.path.dirname(GOLDEN), "..", "tools")
    if tools not in sys.path:
        sys.path.insert(0, tools)
    from chaos_rows import rel

    jobs = [(p, prof, sub, curve, scal) for p in _PERTS]
    if workers > 1:
        import multiprocessing as mp
        from concurrent.futures import ProcessPoolExecutor

        with ProcessPoolExecutor(min(workers, len(jobs)), mp_context=mp.get_context("spawn")) as ex:
            runs = list(ex.map(_oracle_run, jobs))
    else:
        runs = [_oracle_run(j) for j in jobs]
    a, sa = runs[0]
    oka = (sa & 0xFF) == 0
    rmax = np.zeros_like(a)
    for b, sb in runs[1:]:
        okb = (sb & 0xFF) == 0
        r = rel(a, b)
        r[oka != okb] = np.inf
        r[~oka & ~okb] = 0.0
        rmax = np.maximum(rmax, r)
    r = rmax[oka]
    floor = {"moved_1e-5": (r > 1e-5).mean(axis=0).tolist(),
             "moved_1e-3": (r > 1e-3).mean(axis=0).tolist()}
    return a, sa, floor, rmax
