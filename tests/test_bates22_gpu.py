"""GPU parity of pfe_bates22 (C-ABI) against the reference's golden vectors and the oracle.

Bar (SURVEY.md §8(a) parity classes):
  * the failing candidates (reference raised -> row dropped) are exactly the same;
  * s3 (integer peak count), s4, s12-s16, s20, s22: bit-exact on every candidate;
  * every other score j (the class-X fits s1, s2, s19, s21 included) but s10/s11, row by
    row against the golden sets: on every candidate whose
    reference score is stable -- it moves by at most STABLE = 1e-7 relative under each of
    seven ulp-scale perturbations of the fits (start points +-1, +-2, +4 ulp; two patterns
    of +-1 ulp on the residuals: tests/golden/chaos_rows.npz, tools/chaos_rows.py) -- the
    GPU is within 1e-5 of the reference (a row is stable for an output of a fit only if every
    output of that fit is: golden_util.FIT_GROUPS); on the candidates
    where the reference itself moves, the GPU may differ, and the fraction of candidates
    differing by more than 1e-5 (1e-3) is held to 1.5 x the reference's own floor (the
    fraction of candidates moving under the nudges, tests/golden/chaos_floor.json and
    chaos_rows.npz) plus one candidate;
  * every LM score, s10/s11 included, row by row against the reference's own ENVELOPE
    (golden_util.envelope_check, tests/golden/chaos_envelope.npz: per candidate the range of
    K = 50 samples -- the golden value, the oracle's own run, which for s10/s11 is a second
    evaluation in another heap state, and 48 ulp-scale nudges): inside it to 1e-5 on every
    row where the samples agree, and on the chaotic rows outside it no more often than one
    more draw of the same process would be (binomial, p = 2/(K+1));
  * s10/s11 are otherwise held to the population floor: the reference does not reproduce
    ITSELF there -- the same candidate scored twice in one process moves s10/s11 in 4-18% of
    rows (tests/test_oracle_golden.py);
  * fresh (non-golden) batches are checked against the oracle the same way with that
    batch's own perturbation data; the one exception is s9 of the lp = 200 batch, where
    tools/basin_probe.py showed a candidate that is stable under the seven deterministic
    perturbations reaching the GPU's value in the reference itself under per-step ulp noise
    (profiles/r02_basin_probe_lp200.txt): one row allowed there.
"""
import json
import os

import numpy as np
import pytest

from golden_util import (FIT_GROUPS, GOLDEN, SELF_NOISY, bates_inputs, envelope_check, load,
                         oracle_with_floor)
from pulsarfeatureextractor_amd.synth import bates_batch

pytestmark = pytest.mark.gpu

BITEXACT = (2, 3, 11, 12, 13, 14, 15, 19, 21)
STABLE = 1e-7  # a reference score that moves by at most this under every nudge is stable: its
               # value is reproducible to 7 digits, so the GPU is held to 1e-5 there
FLOOR = json.load(open(os.path.join(GOLDEN, "chaos_floor.json")))
ROWS = np.load(os.path.join(GOLDEN, "chaos_rows.npz"))


def rel_err(got, ref):
    with np.errstate(all="ignore"):
        same = (got == ref) | (np.isnan(got) & np.isnan(ref))
        r = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-300)
    r[same] = 0.0
    r[np.isnan(r)] = np.inf
    return r


def check_against(out, st, ref, ref_ok, tag, floor, bitexact=BITEXACT, close=(), rmax=None,
                  stable_slack=0):
    """close: scores held to <= 1e-12 relative instead of bit-exactness -- s20/s22 at lengths
    where numpy's BLAS dot products sum in another order than a power-of-two tree (the
    difference is an ulp).  rmax: (n, 22) per-candidate reference movement under the
    perturbations: row-conditioned parity on the stable candidates, of which stable_slack
    ({score number: rows}) may still differ: only where tools/basin_probe.py showed a
    candidate that is stable under the seven deterministic perturbations changing basin
    under per-step noise in the reference itself (s9 at lp = 200,
    profiles/r02_basin_probe_lp200.txt)."""
    gok = (st & 0xFF) == 0
    assert np.array_equal(gok, ref_ok), f"{tag}: failure pattern differs"
    got, ref = out[gok], ref[gok]
    r = rel_err(got, ref)
    n = max(1, len(r))
    for j in bitexact:
        assert (r[:, j] == 0).all(), f"{tag}: s{j + 1} not bit-exact ({(r[:, j] > 0).sum()} rows)"
    for j in close:
        assert (r[:, j] <= 1e-12).all(), f"{tag}: s{j + 1} max rel {r[:, j].max():.3g} > 1e-12"
    stable = None if rmax is None else rmax[gok] <= STABLE
    if stable is not None:  # a fit is stable on a row only if all of its outputs are
        for grp in FIT_GROUPS:
            both = np.logical_and.reduce([stable[:, j] for j in grp])
            for j in grp:
                stable[:, j] = both
    if rmax is not None:  # the set's own floor over all the nudges, where it is larger
        floor = {key: np.maximum(floor[key], (rmax[gok] > tol).mean(axis=0)).tolist()
                 for tol, key in ((1e-5, "moved_1e-5"), (1e-3, "moved_1e-3"))}
    for j in range(22):
        if j in bitexact or j in close:
            continue
        if stable is not None and j not in SELF_NOISY:
            bad = np.where(stable[:, j] & (r[:, j] > 1e-5))[0]
            if len(bad) and os.environ.get("PFE_PARITY_LOG"):
                with open(os.environ["PFE_PARITY_LOG"], "a") as f:
                    f.write(json.dumps({"tag": tag, "score": j + 1, "rows": bad.tolist(),
                                        "rel": r[bad, j].tolist()}) + "\n")
            allow = stable_slack.get(j + 1, 0) if isinstance(stable_slack, dict) else stable_slack
            assert len(bad) <= allow, (f"{tag}: s{j + 1} beyond 1e-5 on {len(bad)} candidates where "
                                   f"the reference is stable (rows {bad[:10].tolist()})")
        for tol, key in ((1e-5, "moved_1e-5"), (1e-3, "moved_1e-3")):
            moved = (r[:, j] > tol).mean()
            allowed = 1.5 * floor[key][j] + 1.0 / n
            assert moved <= allowed, (f"{tag}: s{j + 1} differs by > {tol} in {moved:.3f} of rows "
                                      f"(reference 1-ulp floor {floor[key][j]:.3f})")


@pytest.mark.parametrize("name", ["bates22_phcx128", "bates22_superb64", "bates22_phcx128_wide"])
def test_vs_reference_golden(engine, name):
    d = load(name)
    prof, sub, curve, scal = bates_inputs(d)
    out, st = engine.bates22(prof, sub, curve, scal)
    assert not (st & 0x10).any(), "PFE_ST_UNSUPPORTED"
    check_against(out, st, d["out"], d["ok"], name, FLOOR.get(name, FLOOR["bates22_phcx128"]),
                  rmax=ROWS[f"{name}_rmax"])
    envelope_check(out, st, name, skip=BITEXACT)


@pytest.mark.parametrize("name", ["bates22_phcx128_big", "bates22_superb64_big"])
def test_vs_reference_golden_big(engine, name):
    """1000 PHCX / 500 SUPERB candidates scored by the reference itself (round 4): the same
    failing candidates, the bit-exact columns exact, and every LM score pinned row by row to
    the reference's own 50-sample envelope (tight rows inside, chaotic rows to the binomial
    bound) -- many more tight rows for s10/s11/s17/s18 than the 300 / 150-row sets."""
    d = load(name)
    prof, sub, curve, scal = bates_inputs(d)
    out, st = engine.bates22(prof, sub, curve, scal)
    assert not (st & 0x10).any(), "PFE_ST_UNSUPPORTED"
    gok = (st & 0xFF) == 0
    assert np.array_equal(gok, d["ok"].astype(bool)), f"{name}: failure pattern differs"
    r = rel_err(out[gok], d["out"][gok])
    for j in BITEXACT:
        assert (r[:, j] == 0).all(), f"{name}: s{j + 1} not bit-exact ({(r[:, j] > 0).sum()} rows)"
    stats = envelope_check(out, st, name, skip=BITEXACT)
    # the reference is reproducible (tight) on 367 / 97 rows of the PHCX set and 48 / 51 of
    # the SUPERB set for s10-s11 / s17-s18 (tools/chaos_envelope.py): all of them were checked
    least = {"bates22_phcx128_big": (360, 90), "bates22_superb64_big": (45, 45)}[name]
    for sc, k in ((10, 0), (11, 0), (17, 1), (18, 1)):
        assert stats[sc][0] >= least[k], f"{name}: only {stats[sc][0]} tight rows for s{sc}"


def test_vs_oracle_fresh_inputs(engine):
    """1000 fresh candidates against the oracle (eight oracle passes in 8 spawned processes)."""
    b = bates_batch(1000, seed=77)
    out, st = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    ref, rst, own, rmax = oracle_with_floor(b["prof"], b["sub"], b["dmcurve"], b["scal"],
                                            workers=8)
    gold = FLOOR["bates22_phcx128"]
    floor = {k: np.maximum(own[k], gold[k]).tolist() for k in gold if k.startswith("moved")}
    check_against(out, st, ref, (rst & 0xFF) == 0, "oracle", floor, rmax=rmax)


@pytest.mark.parametrize("lp,n", [(256, 96), (100, 64), (200, 48), (512, 24)])
def test_vs_oracle_other_lengths(engine, lp, n):
    """Config 4 (Lp = Lsb = 256), ragged lengths (MPL slots partly empty) and the long-profile
    kernels (lp > 256: 16 rows per lane, wide histograms)."""
    b = bates_batch(n, lp=lp, lsb=lp, seed=1000 + lp)
    out, st = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    ref, rst, own, rmax = oracle_with_floor(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    pow2 = lp & (lp - 1) == 0
    exact = BITEXACT if pow2 else tuple(j for j in BITEXACT if j not in (19, 21))
    # floor: the larger of this batch's own 1-ulp floor and the 128-bin golden floor
    gold = FLOOR["bates22_phcx128"]
    floor = {k: np.maximum(own[k], gold[k]).tolist() for k in gold if k.startswith("moved")}
    check_against(out, st, ref, (rst & 0xFF) == 0, f"oracle lp={lp}", floor,
                  bitexact=exact, close=() if pow2 else (19, 21), rmax=rmax,
                  stable_slack={9: 1} if lp == 200 else 0)


def lm_columns_agree(o0, s0, o1, s1, floor, slack=0.03, tag=""):
    """Two GPU solvers on the same candidates: same failures, the bit-exact columns
    identical, the LM columns different by > 1e-5 on no more rows than 1.5 x the reference's
    own 1-ulp floor for that profile length + `slack` (both solvers sum their m-rows in
    another order than MINPACK and contract the solver's linear algebra into FMAs, so on
    the chaotic rows each lands on one of the reference's own nearby values)."""
    assert np.array_equal(s0, s1), tag
    ok = (s0 & 0xFF) == 0
    r = rel_err(o1[ok], o0[ok])
    for j in BITEXACT:
        assert (r[:, j] == 0).all(), f"{tag} s{j + 1}"
    for j in range(22):
        if j not in BITEXACT:
            moved = (r[:, j] > 1e-5).mean()
            assert moved <= 1.5 * floor["moved_1e-5"][j] + slack, f"{tag} s{j + 1}: {moved:.3f}"


def floor_for(lp):
    """The reference's 1-ulp chaos floor of the golden set nearest in profile length."""
    return FLOOR["bates22_superb64"] if lp <= 64 else FLOOR["bates22_phcx128"]


def test_batched_solver_matches_wave_solver(engine):
    """The batched lmdif kernels (lm_batch.h) against the wave-per-fit kernels (handle option
    solver = wave / batched).  Without FMA contraction of the solver's linear algebra
    (libpfe_nofma builds) the two are bit-identical; with it, the compiler contracts each
    inlined code shape on its own, so they are held to lm_columns_agree."""
    b = bates_batch(200, seed=21)
    with engine.options(solver="wave"):
        o0, s0 = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    with engine.options(solver="batched"):
        o1, s1 = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    lm_columns_agree(o0, s0, o1, s1, floor_for(128), tag="wave vs batched")


@pytest.mark.parametrize("solver", ["wave", "batched"])
def test_every_solver_inside_reference_envelope(engine, solver):
    """The determinism guard between the GPU solvers that the FMA-contracted linear algebra
    took from bit identity: each non-default solver, like the pooled default
    (test_vs_reference_golden), holds every tight row of the reference's own 50-sample
    envelope and the binomial bound on the chaotic rows, with the bit-exact columns exact --
    so a real divergence in one solver fails on the rows where the reference is
    reproducible, with no slack."""
    d = load("bates22_phcx128")
    prof, sub, curve, scal = bates_inputs(d)
    with engine.options(solver=solver):
        out, st = engine.bates22(prof, sub, curve, scal)
    gok = (st & 0xFF) == 0
    assert np.array_equal(gok, d["ok"].astype(bool)), solver
    r = rel_err(out[gok], d["out"][gok])
    for j in BITEXACT:
        assert (r[:, j] == 0).all(), f"{solver}: s{j + 1}"
    envelope_check(out, st, "bates22_phcx128", skip=BITEXACT)


def test_concurrent_groups_and_hand_over_bit_identical(engine):
    """The score groups on side streams (default) vs in order on one stream (option
    serial=1), the LM hand-over of accepted residuals (default) vs re-evaluation
    (handover=0), and the pool size (gslots): the same bits (tests/test_pfd22_gpu.py checks
    the PFD path)."""
    b = bates_batch(300, seed=33)
    ref = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    for env in ({"serial": 1}, {"handover": 0}, {"serial": 1, "handover": 0}, {"gslots": 7}):
        with engine.options(**env):
            o, s = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
        assert np.array_equal(s, ref[1]), env
        assert np.array_equal(np.nan_to_num(o, nan=7.0), np.nan_to_num(ref[0], nan=7.0)), env


def test_device_pointers_and_determinism(engine):
    import torch

    b = bates_batch(256, seed=5)
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in b.items()}
    o1, s1 = engine.bates22(t["prof"], t["sub"], t["dmcurve"], t["scal"])
    o2, s2 = engine.bates22(t["prof"], t["sub"], t["dmcurve"], t["scal"])
    engine.synchronize()
    assert torch.equal(s1, s2)
    assert torch.equal(torch.nan_to_num(o1, 7.0), torch.nan_to_num(o2, 7.0))
    h, hs = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    assert np.array_equal(np.nan_to_num(h, nan=7.0), np.nan_to_num(o1.cpu().numpy(), nan=7.0))


def test_batch_independence(engine):
    """A candidate's scores do not depend on its neighbours (shard/concat equivalence)."""
    b = bates_batch(96, seed=9)
    full, sf = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    for cuts in ((0, 32, 64, 96), (0, 7, 40, 41, 96)):  # whole and partial 32-fit batches
        parts = [engine.bates22(b["prof"][i:j], b["sub"][i:j], b["dmcurve"][i:j], b["scal"][i:j])
                 for i, j in zip(cuts[:-1], cuts[1:])]
        cat = np.concatenate([p[0] for p in parts])
        assert np.array_equal(np.nan_to_num(cat, nan=7.0), np.nan_to_num(full, nan=7.0))


@pytest.mark.parametrize("lp,n", [(128, 600), (64, 600), (256, 300), (200, 200)])
def test_pooled_group_solver(engine, lp, n):
    """The pooled group-LM kernels (lm_group.h, the default for <= 256 bins: 16-lane groups up
    to 128 bins, 32-lane groups above) against the batched wave kernels: same failures,
    bit-exact columns identical, the LM outputs different only in the last bits of their
    m-sums (so at most at the reference's own 1-ulp chaos rates), and every fit's result
    independent of the pool it ran in."""
    b = bates_batch(n, lp=lp, lsb=lp, seed=33 + lp)
    with engine.options(solver="batched"):
        o0, s0 = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    o1, s1 = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    lm_columns_agree(o0, s0, o1, s1, floor_for(lp), tag=f"pooled vs batched lp={lp}")
    # pool independence: the same candidates in another order and batch size
    perm = np.random.default_rng(1).permutation(len(b["prof"]))[:n * 5 // 12]
    o2, s2 = engine.bates22(b["prof"][perm], b["sub"][perm], b["dmcurve"][perm], b["scal"][perm])
    assert np.array_equal(s2, s1[perm])
    assert np.array_equal(np.nan_to_num(o2, nan=7.0), np.nan_to_num(o1[perm], nan=7.0))


def wide_histogram_batch(n, seed):
    """Profiles with low noise under a strong narrow pulse: Freedman-Diaconis bin counts of
    ~40 (pooled kernels), ~100-190 (deferred to the wave kernel, > 64 bins), ~350-390
    (the 1024-bin wave kernel, > 256 bins) and, from quantised sigma ~ 0.5 noise, often
    1000-1600 (k_ghist_wide, rows in global scratch)."""
    b = bates_batch(n, seed=seed)
    rng = np.random.default_rng(seed)
    lp = b["prof"].shape[1]
    x = np.arange(lp)
    prof = np.empty((n, lp))
    for i in range(n):
        kind = i % 4
        sd = (2.5, 0.7, 6.0, 0.5)[kind]
        base = rng.normal(100 if kind != 1 else 50, sd, lp)
        mu, w = rng.uniform(10, lp - 10), rng.uniform(1.0, 3.0)
        prof[i] = base + 150 * np.exp(-0.5 * ((x - mu) / w) ** 2)
    b["prof"] = np.clip(np.rint(prof), 0, 255).astype(np.uint8)
    return b


def test_wide_histograms_vs_oracle(engine):
    """Every histogram-width class in one batch: the pooled kernels take <= 64 bins and pass
    wider ones on (ST_DEFER_HIST64, ST_DEFER_HIST, ST_DEFER_WIDE); all of them against the
    oracle, none left unscored."""
    from oracle.bates import backward_diff, fd_bins

    b = wide_histogram_batch(80, 5)
    widest = max(max(fd_bins(p.astype(np.int64)), fd_bins(backward_diff(p.astype(np.int64))))
                 for p in b["prof"])
    assert widest > 1024, widest
    out, st = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    assert not (st & 0xFFFF0000).any(), "internal deferral bits left in status"
    assert not (st & 0x10).any(), "PFE_ST_UNSUPPORTED"
    ref, rst, own, rmax = oracle_with_floor(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    gold = FLOOR["bates22_phcx128"]
    floor = {k: np.maximum(own[k], gold[k]).tolist() for k in gold if k.startswith("moved")}
    check_against(out, st, ref, (rst & 0xFF) == 0, "wide histograms", floor, rmax=rmax)


def test_pooled_tiny_and_empty_batches(engine):
    """Pools with fewer candidates than slots (1, 3, 33 rows) give every candidate the scores
    it gets in a large batch; an empty batch is a no-op."""
    b = bates_batch(200, seed=41)
    full, sf = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    for k in (1, 3, 33):
        o, s = engine.bates22(b["prof"][:k], b["sub"][:k], b["dmcurve"][:k], b["scal"][:k])
        assert np.array_equal(s, sf[:k])
        assert np.array_equal(np.nan_to_num(o, nan=7.0), np.nan_to_num(full[:k], nan=7.0)), k
    o, s = engine.bates22(b["prof"][:0], b["sub"][:0], b["dmcurve"][:0], b["scal"][:0])
    assert o.shape == (0, 22) and s.shape == (0,)


def test_config3_full_size_10m(engine):
    """BASELINE config 3 at the size it names: pfe_bates22 over 10M resident candidates (one
    16384-candidate synthetic block tiled, as bench.py's extra.config3 does).  Every tile's
    scores and status must be the bits of the first tile (a work-queue or 32-bit indexing
    fault past a few million rows would break that), and the first 300 rows must meet the
    fresh-batch oracle bar."""
    import torch

    n, blk = 10_000_000, 16384
    b = bates_batch(blk, seed=20261018)
    reps = (n + blk - 1) // blk
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda()
         .repeat((reps,) + (1,) * (v.ndim - 1))[:n].contiguous() for k, v in b.items()}
    out, st = engine.bates22(t["prof"], t["sub"], t["dmcurve"], t["scal"])
    engine.synchronize()
    del t
    full = (n // blk) * blk
    ob = out.view(torch.int64)
    tiles = ob[:full].view(-1, blk, 22)
    bad = (tiles != tiles[:1]).any(dim=2).any(dim=1)
    assert not bool(bad.any()), f"tiles differing from tile 0: {torch.nonzero(bad)[:10].flatten().tolist()}"
    sv = st[:full].view(-1, blk)
    assert bool((sv == sv[:1]).all()), "status differs between tiles"
    assert torch.equal(ob[full:], ob[: n - full]) and torch.equal(st[full:], st[: n - full])
    k = 300
    o0, s0 = out[:k].cpu().numpy(), st[:k].cpu().numpy().astype(np.uint32)
    del out, st, ob, tiles, sv
    torch.cuda.empty_cache()
    ref, rst, own, rmax = oracle_with_floor(b["prof"][:k], b["sub"][:k], b["dmcurve"][:k],
                                            b["scal"][:k], workers=8)
    gold = FLOOR["bates22_phcx128"]
    floor = {kk: np.maximum(own[kk], gold[kk]).tolist() for kk in gold if kk.startswith("moved")}
    check_against(o0, s0, ref, (rst & 0xFF) == 0, "config 3 @10M, tile 0", floor, rmax=rmax)
