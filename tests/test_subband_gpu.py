"""GPU parity of the sub-band scores (s20-s22; pfe_subband3 and columns 19-21 of pfe_bates22)
against the oracle (oracle/bates.subband_scores, the restatement of
ProfileOperations.getSubband_scores :1585-1686 and PHCXOperations.getProfileCorr :387-415)
and against the reference's own golden sets.

Bar: identical failing candidates; s20 (integer boxcar maxima) bit-exact; s22 bit-exact at
64/128/256 bins (numpy's BLAS dot order) and within 1e-12 elsewhere; s21 -- computed from
exact integer boxcar moments through sum_{i<k} cc_ik = (|sum_i z_i|^2 - sum_i |z_i|^2) / 2
instead of the reference's pair loop -- within 1e-9 relative (north_star: 1e-5).
"""
import numpy as np
import pytest

from golden_util import bates_inputs, load
from oracle.bates import subband_scores
from pulsarfeatureextractor_amd.synth import bates_batch

pytestmark = pytest.mark.gpu


def oracle_sub(prof, sub, scal):
    n = len(prof)
    out = np.full((n, 3), np.nan)
    ok = np.zeros(n, dtype=bool)
    import warnings

    with warnings.catch_warnings(), np.errstate(all="ignore"):
        warnings.simplefilter("ignore")
        for i in range(n):
            try:
                if prof.shape[1] != sub.shape[2]:
                    raise ValueError("corrcoef: all the input array dimensions must match")
                out[i] = subband_scores(np.asarray(sub[i], dtype=np.int64),
                                        np.asarray(prof[i], dtype=np.int64), float(scal[i, 3]))
                ok[i] = True
            except Exception:
                pass
    return out, ok


def rel(a, b):
    with np.errstate(all="ignore"):
        r = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    r[(a == b) | (np.isnan(a) & np.isnan(b))] = 0.0
    r[np.isnan(r)] = np.inf
    return r


def check(out, st, ref, ok, tag, lsb):
    gok = (st & 0xFF) == 0
    assert np.array_equal(gok, ok), f"{tag}: failure pattern differs at {np.where(gok != ok)[0][:10]}"
    assert not (st & 0x10).any(), f"{tag}: PFE_ST_UNSUPPORTED set"
    r = rel(out[ok], ref[ok])
    assert (r[:, 0] == 0).all(), f"{tag}: s20 not bit-exact ({(r[:, 0] > 0).sum()} rows)"
    assert (r[:, 1] <= 1e-9).all(), f"{tag}: s21 max rel {r[:, 1].max():.3g}"
    if lsb in (64, 128, 256):
        assert (r[:, 2] == 0).all(), f"{tag}: s22 not bit-exact (max rel {r[:, 2].max():.3g})"
    else:
        assert (r[:, 2] <= 1e-12).all(), f"{tag}: s22 max rel {r[:, 2].max():.3g}"


def adversarial(b):
    """Rows the reference fails or treats specially."""
    sub, scal = b["sub"], b["scal"]
    lsb = sub.shape[2]
    sub[0] = 0                        # every pair NaN: m = 0 -> ZeroDivisionError
    scal[1, 3] = 0.0                  # wb = 0: rms = stdev / 0
    scal[2, 3] = 2.0                  # wb > nBins: no window, max_bin unbound
    scal[3, 3] = np.nan               # int(ceil(nan)) raises
    sub[4, 1:] = 7                    # one varying band: no valid pair
    sub[5, sub.shape[1] - 1] = 9      # a constant band among varying ones: its pairs skipped
    sub[6, :, :] = sub[6, :1, :]      # identical bands: cc = 1 (clipped)
    scal[7, 3] = 1.0 / lsb            # wb = 1
    scal[8, 3] = 1.0                  # wb = nBins: one window per band
    return b


@pytest.mark.parametrize("nsub,lsb,n", [(16, 64, 48), (16, 128, 48), (16, 256, 40), (32, 128, 24),
                                        (64, 64, 20), (40, 100, 16), (3, 1024, 12), (24, 200, 12),
                                        (2, 16, 24), (5, 37, 24)])
def test_subband3_vs_oracle(engine, nsub, lsb, n):
    b = adversarial(bates_batch(n, lp=lsb, nsub=nsub, lsb=lsb, seed=500 + nsub + lsb))
    out, st = engine.subband3(b["prof"], b["sub"], b["scal"])
    ref, ok = oracle_sub(b["prof"], b["sub"], b["scal"])
    check(out, st, ref, ok, f"{nsub}x{lsb}", lsb)


@pytest.mark.parametrize("nsub,lsb", [(16, 64), (16, 128), (16, 256), (24, 200), (8, 512)])
def test_subband3_bright_wide_windows(engine, nsub, lsb):
    """Boxcar sums past 46 341 (b^2 >= 2^31): bright bands (bytes 180-255) and windows of
    70-100 % of the band, so every sum of squares sits in the top bit of 32 bits or beyond."""
    n = 24
    b = bates_batch(n, lp=lsb, nsub=nsub, lsb=lsb, seed=900 + lsb)
    rng = np.random.default_rng(lsb)
    b["sub"][:] = rng.integers(180, 256, size=b["sub"].shape, dtype=np.uint8)
    b["sub"][:, :, : lsb // 4] = 255
    b["scal"][:, 3] = rng.uniform(0.7, 0.98, size=n)
    out, st = engine.subband3(b["prof"], b["sub"], b["scal"])
    ref, ok = oracle_sub(b["prof"], b["sub"], b["scal"])
    assert ok.all()
    check(out, st, ref, ok, f"bright {nsub}x{lsb}", lsb)


@pytest.mark.parametrize("nsub,lsb", [(16, 256), (20, 128), (16, 64), (3, 32)])
def test_subband3_packed_pass_boundary(engine, nsub, lsb):
    """The fast kernel's packed pass 1 (two windows per register, wb <= 32; 16-pair chunks
    for wb <= 16) at its bounds:
    windows of 29-36 bins (both parities, both sides of 32) and 1-3 bins, saturated bands
    (every byte 255: b = 255 wb, the largest the packed keys and 32-bit square sums hold),
    random bright bands and ties between equal windows."""
    wbs = [w for w in (1, 2, 3, 15, 16, 17, 29, 30, 31, 32, 33, 34, 36) if w <= lsb]
    n = 4 * len(wbs)
    b = bates_batch(n, lp=lsb, nsub=nsub, lsb=lsb, seed=1300 + lsb)
    rng = np.random.default_rng(1400 + lsb)
    for i in range(n):
        b["scal"][i, 3] = wbs[i % len(wbs)] / lsb  # exact: ceil(w * lsb) = wb
        kind = i // len(wbs)
        if kind == 0:
            b["sub"][i] = 255
            b["sub"][i, :, 0] = rng.integers(0, 256, size=nsub)  # keep the bands varying
        elif kind == 1:
            b["sub"][i] = rng.integers(200, 256, size=b["sub"][i].shape, dtype=np.uint8)
        elif kind == 2:
            b["sub"][i] = 0
            b["sub"][i, :, ::8] = 255                              # periodic: tied windows
            b["sub"][i, :, 1] = rng.integers(0, 256, size=nsub)
    out, st = engine.subband3(b["prof"], b["sub"], b["scal"])
    ref, ok = oracle_sub(b["prof"], b["sub"], b["scal"])
    check(out, st, ref, ok, f"packed {nsub}x{lsb}", lsb)


def test_subband3_matches_bates22_columns_and_device(engine):
    import torch

    b = adversarial(bates_batch(64, seed=8))
    o3, s3 = engine.subband3(b["prof"], b["sub"], b["scal"])
    o22, s22 = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    ok3 = (s3 & 0xFF) == 0
    assert np.array_equal(ok3, (s22 & 0x08) == 0)
    assert np.array_equal(o3[ok3], o22[ok3][:, 19:22])
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in b.items()}
    od, sd = engine.subband3(t["prof"], t["sub"], t["scal"])
    engine.synchronize()
    assert np.array_equal(sd.cpu().numpy().view(np.uint32), s3)
    assert np.array_equal(np.nan_to_num(od.cpu().numpy(), nan=7.0), np.nan_to_num(o3, nan=7.0))


def test_config4_literal_shape_fails_like_the_reference(engine):
    """BASELINE config 4 as worded (256-bin profile, 16 x 128 sub-bands): the reference's
    getProfileCorr correlates 128-bin bands with the 256-bin profile and numpy raises, so
    every candidate fails in its sub-band group (golden set made by the reference itself);
    the other 19 scores are still computed and match the oracle's groups."""
    d = load("bates22_cfg4_256x128")
    assert not d["ok"].any()
    prof, sub, curve, scal = bates_inputs(d)
    out, st = engine.bates22(prof, sub, curve, scal)
    assert ((st & 0x08) != 0).all(), np.unique(st & 0xFF)
    # the reference names the first group that raised: the sub-band group, except where the
    # Gaussian group raised before it
    gauss = np.array(["Gaussian" in e for e in d["err"]])
    assert np.array_equal((st & 0x02) != 0, gauss)
    o3, s3 = engine.subband3(prof, sub, scal)
    assert ((s3 & 0xFF) == 0x08).all()
    # the other groups against the oracle's per-group restatement
    import warnings

    from oracle import bates as ob

    with warnings.catch_warnings(), np.errstate(all="ignore"):
        warnings.simplefilter("ignore")
        for i in range(len(prof)):
            p = np.asarray(prof[i], dtype=np.int64)
            try:
                ref = ob.sinusoid_scores(p)
            except Exception:
                continue
            r = rel(out[i, :4], np.asarray(ref, dtype=np.float64))
            assert r[2] == 0 and r[3] == 0, i                                # s3, s4 bit-exact
            assert r[0] <= 1e-5, i
            par = ob.parameter_scores(scal[i])
            assert np.array_equal(out[i, 11:15], par), i                    # s12-s15 bit-exact


def test_nsub32_vs_reference_golden(engine):
    """32 sub-bands (nSub read from the file): the reference's own scores."""
    d = load("bates22_phcx128_nsub32")
    prof, sub, curve, scal = bates_inputs(d)
    assert sub.shape[1] == 32
    o3, s3 = engine.subband3(prof, sub, scal)
    ref = d["out"]
    ok = d["ok"]
    gok = (s3 & 0xFF) == 0
    # the reference fails a candidate for any group; the sub-band group alone must not fail
    # where the reference scored the candidate
    assert gok[ok].all()
    r = rel(o3[ok], ref[ok][:, 19:22])
    assert (r[:, 0] == 0).all() and (r[:, 2] == 0).all() and (r[:, 1] <= 1e-9).all(), r.max(axis=0)
    out, st = engine.bates22(prof, sub, curve, scal)
    assert np.array_equal((st & 0xFF) == 0, ok)


@pytest.mark.parametrize("nsub,lsb,n", [(32, 1024, 10), (64, 512, 10), (300, 8, 10), (1, 64, 4),
                                        (12, 1500, 4), (4, 3000, 3)])
def test_any_shape_subband_vs_oracle(engine, nsub, lsb, n):
    """Sub-band shapes the LDS-resident kernels do not hold (nsub > 256, nsub (nBins + 1) >
    32768, nBins > 1024, nsub = 1) through the global-scratch kernel (k_subband_g): the
    reference scores any shape, so these are parity tests against the oracle -- pfe_subband3
    and columns 19-21 of pfe_bates22 (where lp = nBins fits the 22-score kernels), adversarial
    rows included.  Windows of <= 10 % keep the oracle's pure-Python boxcar loop short."""
    b = bates_batch(n, lp=min(lsb, 1024), nsub=16, lsb=min(lsb, 1024), seed=600 + nsub + lsb)
    rng = np.random.default_rng(nsub * 7 + lsb)
    sub = rng.integers(0, 256, (n, nsub, lsb), dtype=np.uint8)
    sub[:, :, lsb // 3: lsb // 3 + max(1, lsb // 20)] += 40  # a common bright window
    prof = rng.integers(0, 256, (n, lsb), dtype=np.uint8)
    scal = b["scal"].copy()
    scal[:, 3] = rng.uniform(0.5 / lsb, 0.1, size=n)
    b2 = {"sub": sub, "scal": scal}
    if n >= 9:
        b2 = adversarial(b2)
    out, st = engine.subband3(prof, b2["sub"], b2["scal"])
    ref, ok = oracle_sub(prof, b2["sub"], b2["scal"])
    check(out, st, ref, ok, f"{nsub}x{lsb}", lsb)
    if lsb <= 1024 and lsb >= 8:
        o22, s22 = engine.bates22(prof, b2["sub"], b["dmcurve"], b2["scal"])
        assert not (s22 & 0x10).any()
        assert np.array_equal((s22 & 0x08) == 0, ok)
        assert np.array_equal(o22[ok][:, 19:22], out[ok])


def test_subband_shape_beyond_every_kernel_fails_rows_not_call(engine):
    """nsub > 65536: pfe_bates22 marks every row PFE_ST_UNSUPPORTED and still computes the
    other score groups exactly as for the same candidates with an ordinary sub-band shape;
    pfe_subband3 (nothing else to compute) refuses the call."""
    from pulsarfeatureextractor_amd._native import PfeError

    b = bates_batch(8, lp=128, nsub=16, lsb=128, seed=77)
    big = np.random.default_rng(3).integers(0, 256, (8, 65537, 2), dtype=np.uint8)
    ref, rst = engine.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    o, st = engine.bates22(b["prof"], big, b["dmcurve"], b["scal"])
    assert ((st & 0x10) != 0).all()
    assert np.array_equal(st & ~np.uint32(0x18), rst & ~np.uint32(0x18))
    assert np.array_equal(o[:, :19], ref[:, :19], equal_nan=True)
    with pytest.raises(PfeError):
        engine.subband3(b["prof"], big, b["scal"])


def test_config4_full_size_1m(engine):
    """BASELINE config 4 at the size it names and bench.py times (extra.config4): one
    pfe_subband3 launch over 1M resident candidates of a 256-bin profile and 16 x 256
    sub-bands, on device pointers.
      * bench.py's rows (its 16384-row block, seed 20261021, tiled to 1M): every tile's scores
        and status bit-identical to the first; the first 100 rows against the oracle;
      * a fresh (untiled) 1M batch generated on the device: 200 rows drawn from the last
        100k against the oracle, s20 and s22 bit-exact, s21 within 1e-9."""
    import torch
    from pulsarfeatureextractor_amd.synth import lyon_batch_torch

    n, blk, lsb = 1_000_000, 16384, 256
    base = bates_batch(blk, lp=lsb, nsub=16, lsb=lsb, seed=20261021)   # bench.py tile_bates
    reps = (n + blk - 1) // blk
    t = {k: torch.from_numpy(np.ascontiguousarray(base[k])).cuda() for k in ("prof", "sub", "scal")}
    bt = {k: v.repeat((reps,) + (1,) * (v.dim() - 1))[:n].contiguous() for k, v in t.items()}
    out, st = engine.subband3(bt["prof"], bt["sub"], bt["scal"])
    engine.synchronize()
    full = (n // blk) * blk
    ob = out.view(torch.int64)
    tiles = ob[:full].view(-1, blk, 3)
    bad = (tiles != tiles[:1]).any(dim=2).any(dim=1)
    assert not bool(bad.any()), f"tiles differing from tile 0: {torch.nonzero(bad)[:10].flatten().tolist()}"
    assert torch.equal(ob[full:], ob[: n - full])
    stt = st[:full].view(-1, blk)
    assert bool((stt == stt[:1]).all()) and torch.equal(st[full:], st[: n - full])
    ref, ok = oracle_sub(base["prof"][:100], base["sub"][:100], base["scal"][:100])
    check(out[:100].cpu().numpy(), st[:100].cpu().numpy().view(np.uint32), ref, ok,
          "config4 tile 0", lsb)
    del out, st, ob, tiles, bt, t
    torch.cuda.empty_cache()
    prof, rows = lyon_batch_torch(n, lsb, 16 * lsb, seed=20261025)
    sub = rows.view(n, 16, lsb)
    g = torch.Generator(device="cuda")
    g.manual_seed(20261026)
    scal = torch.zeros((n, 8), dtype=torch.float64, device="cuda")
    scal[:, 3] = torch.rand(n, generator=g, device="cuda", dtype=torch.float64) * 0.08 + 0.02
    out, st = engine.subband3(prof, sub, scal)
    engine.synchronize()
    idx = torch.randint(n - 100_000, n, (200,), generator=torch.Generator().manual_seed(13))
    pi, si, ci = (x[idx].cpu().numpy() for x in (prof, sub, scal))
    ref, ok = oracle_sub(pi, si, ci)
    check(out[idx].cpu().numpy(), st[idx].cpu().numpy().view(np.uint32), ref, ok,
          "config4 fresh", lsb)
    del out, st, prof, rows, sub, scal
    torch.cuda.empty_cache()
