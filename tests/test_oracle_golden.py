"""Pin the oracle against the reference's own outputs (tests/golden, tools/make_golden.py).

The reference has no tests or fixtures of its own, so these vectors -- the
reference itself run on synthetic PHCX/SUPERB files -- are the pin.

Bar:
  * Lyon-8: bit-exact (same numpy/scipy calls on the same rows).
  * Bates-22: same failing candidates; bit-exact on every score but s10/s11 on the original
    sets, and outside class C (the LM outputs s7-s11, s17, s18) on the round-4 big sets, where
    the class-C scores are bit-exact on the rows the reference's envelope calls tight; all
    LM scores inside the reference's own 50-sample envelope, s10/s11
    also within 1e-5 relative of the golden draw in >= 70% of rows, the others in >= 90%.  The reference is not bit-reproducible against
    ITSELF on s10/s11: the same candidate scored twice in one process (different heap state)
    moves s10/s11 in 4-18% of rows (last-bit differences inside numpy/MINPACK that the
    8-pass double-Gaussian peel amplifies; measured), so no golden vector can
    pin those two scores more tightly.
"""
import numpy as np
import pytest

from golden_util import (CLASS_C, ENVELOPE_TIGHT, FIT_GROUPS, GOLDEN, SELF_NOISY, bates_inputs,
                         envelope_check, load)
from oracle.bates import bates22
from oracle.lyon import lyon8


@pytest.mark.parametrize("name", ["lyon8_superb64", "lyon8_phcx128", "lyon8_phcx128_dmplane"])
def test_lyon8_oracle_bit_exact(name):
    d = load(name)
    assert d["ok"].all()
    got = lyon8(d["prof"], d["block0"])
    ref = d["out"]
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    m = ~np.isnan(ref)
    assert np.array_equal(got[m], ref[m])


def envelope_tight(name):
    """(n, 22) rows where the reference's 50 samples agree to ENVELOPE_TIGHT on a score and on
    every other output of the same fit (golden_util.envelope_check's rule)."""
    import os

    env = np.load(os.path.join(GOLDEN, "chaos_envelope.npz"))
    lo, hi = env[f"{name}_lo"], env[f"{name}_hi"]
    with np.errstate(all="ignore"):
        t = (hi - lo) <= ENVELOPE_TIGHT * np.maximum(np.abs(lo), np.abs(hi))
    t |= np.isnan(lo) & np.isnan(hi)
    for grp in FIT_GROUPS:
        both = np.logical_and.reduce([t[:, j] for j in grp])
        for j in grp:
            t[:, j] = both
    return t


@pytest.mark.parametrize("name,rows", [("bates22_phcx128", 90), ("bates22_superb64", 45),
                                       ("bates22_phcx128_wide", 20),
                                       ("bates22_phcx128_big", 40), ("bates22_superb64_big", 30)])
def test_bates22_oracle_vs_reference(name, rows):
    d = load(name)
    prof, sub, curve, scal = bates_inputs(d)
    ok = d["ok"]
    # every failing row plus a prefix of the set
    sel = np.unique(np.concatenate([np.arange(rows), np.where(~ok)[0]]))
    out, st = bates22(prof[sel], sub[sel], curve[sel], scal[sel])
    assert np.array_equal((st & 0xFF) == 0, ok[sel]), "failure pattern differs"
    m = ok[sel]
    ref = d["out"][sel][m]
    got = out[m]
    same = (got == ref) | (np.isnan(got) & np.isnan(ref))
    with np.errstate(all="ignore"):
        close = same | (np.abs(got - ref) <= 1e-5 * np.abs(ref))
    # bit-exact: every score but s10/s11 on the original sets (round 1-3, made where the
    # oracle reproduced the reference); on the 1000 / 500-row sets of round 4 the class-C fits
    # only where the reference's own 50-sample envelope is tight -- a chaotic row of s7-s9,
    # s17, s18 can land on another of the reference's values
    big = name.endswith("_big")
    tight = envelope_tight(name)[sel][m]
    for j in range(22):
        if j in SELF_NOISY:
            continue
        must = np.ones(len(got), dtype=bool) if (j not in CLASS_C or not big) else tight[:, j]
        bad = must & ~same[:, j]
        assert not bad.any(), f"s{j + 1} not bit-exact in {bad.sum()} rows"
    # the LM outputs (class C): the oracle's draw inside the reference's envelope (tight rows
    # all, chaotic rows to the binomial bound) -- on the larger sets a chaotic row can move
    # s8 or s17 between two runs of the oracle itself; the 70% single-draw agreement of
    # s10/s11 where no envelope row decides
    full = np.full(d["out"].shape, np.nan)
    full[sel] = out
    fst = np.ones(len(ok), dtype=np.int64)
    fst[sel] = st
    stats = envelope_check(full, fst, name, skip=[j for j in range(22) if j not in CLASS_C])
    for j in CLASS_C:
        if j not in SELF_NOISY:
            assert close[:, j].mean() >= 0.90, f"s{j + 1}: {close[:, j].mean():.3f}"
    for j in SELF_NOISY:
        tight_rows, wide_rows = stats[j + 1][0], stats[j + 1][1]
        if tight_rows + wide_rows == 0:
            assert close[:, j].mean() >= 0.70, f"s{j + 1}: {close[:, j].mean():.3f}"


def test_bates22_oracle_vs_reference_nsub32():
    """32 sub-bands per candidate (nSub from the file)."""
    d = load("bates22_phcx128_nsub32")
    prof, sub, curve, scal = bates_inputs(d)
    sel = np.arange(30)
    out, st = bates22(prof[sel], sub[sel], curve[sel], scal[sel])
    ok = d["ok"][sel]
    assert np.array_equal((st & 0xFF) == 0, ok)
    ref = d["out"][sel][ok]
    got = out[ok]
    for j in (19, 20, 21):
        assert np.array_equal(got[:, j], ref[:, j]), f"s{j + 1}"


def test_config4_literal_shape_oracle_fails_like_reference():
    """256-bin profile with 16 x 128 sub-bands: every candidate fails (sub-band group, or the
    Gaussian group first on the constant-profile row)."""
    d = load("bates22_cfg4_256x128")
    prof, sub, curve, scal = bates_inputs(d)
    sel = np.arange(8)
    out, st = bates22(prof[sel], sub[sel], curve[sel], scal[sel])
    assert not d["ok"][sel].any()
    gauss = np.array(["Gaussian" in e for e in d["err"][sel]])
    assert np.array_equal((st & 0xFF) == 0x02, gauss)
    assert ((st & 0xFF)[~gauss] == 0x08).all()


def test_all30_oracle_vs_reference():
    """Config 5's 30 values: Lyon features of the profile + section-0 DataBlock, then the 22
    scores of the same file."""
    d = load("all30_phcx128")
    prof, sub, curve, scal = bates_inputs(d)
    sel = np.arange(20)
    l8 = lyon8(prof[sel], d["block0"][sel])
    out, st = bates22(prof[sel], sub[sel], curve[sel], scal[sel])
    ok = d["ok"][sel]
    assert np.array_equal((st & 0xFF) == 0, ok)
    ref = d["out"][sel][ok]
    assert np.array_equal(l8[ok], ref[:, :8])
    for j in range(22):
        if j not in SELF_NOISY:
            g, r = out[ok][:, j], ref[:, 8 + j]
            assert np.array_equal(g, r) or np.array_equal(np.isnan(g), np.isnan(r)) and \
                np.array_equal(g[~np.isnan(g)], r[~np.isnan(r)]), f"s{j + 1}"
