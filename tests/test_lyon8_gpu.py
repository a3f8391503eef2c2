"""GPU parity: pfe_lyon8_u8 / pfe_lyon8_f64 (C-ABI) vs the oracle restatement.

Tolerances (north_star: 1e-5 relative for the floating-point moments):
  * mean / std: bit-exact for power-of-two row lengths (numpy's sums are exact there and
    the kernel's integer sums are exact everywhere);
  * skew / kurt: |gpu - oracle| <= 1e-12 * max(1, |oracle|) (a few ulp; the kernel
    computes the exact rational moments, numpy rounds d^4 terms);
  * NaN exactly where the oracle has NaN (zero-variance rows).
"""
import numpy as np
import pytest

from oracle.lyon import lyon8, lyon8_batched
from pulsarfeatureextractor_amd.synth import lyon_batch

pytestmark = pytest.mark.gpu
TOL = 1e-12


def check(got, ref, exact_cols=(0, 1, 4, 5)):
    assert got.shape == ref.shape
    assert np.array_equal(np.isnan(got), np.isnan(ref)), "NaN pattern differs"
    m = ~np.isnan(ref)
    err = np.abs(got - ref)[m] / np.maximum(1.0, np.abs(ref[m]))
    assert err.max(initial=0.0) <= TOL, f"max rel err {err.max()}"
    for c in exact_cols:
        g, r = got[:, c], ref[:, c]
        mm = ~np.isnan(r)
        assert np.array_equal(g[mm], r[mm]), f"column {c} not bit-exact"


@pytest.mark.parametrize("L", [64, 128, 256])
def test_fast_path_vs_oracle(engine, L):
    prof, dm = lyon_batch(3000, L, L, seed=100 + L)
    got = engine.lyon8(prof, dm)
    check(got, lyon8(prof, dm))


@pytest.mark.parametrize("lp,ld", [(128, 15360), (100, 37), (1, 1), (2, 3), (64, 128), (257, 1000)])
def test_generic_path_vs_oracle(engine, lp, ld):
    prof, dm = lyon_batch(200, lp, ld, seed=7 + lp + ld, adversarial=lp > 8 and ld > 8)
    got = engine.lyon8(prof, dm)
    exact = (0, 1, 4, 5) if lp in (64, 128, 256) and ld in (64, 128, 256) else (0,)
    check(got, lyon8_batched(prof, dm), exact_cols=exact)


def test_strided_and_unaligned_rows(engine):
    prof, dm = lyon_batch(500, 128, 128, seed=11)
    big = np.zeros((500, 160), dtype=np.uint8)
    big[:, 3:131] = prof
    got = engine.lyon8(big[:, 3:131], dm)  # non-16B-aligned rows -> generic path
    check(got, lyon8(prof, dm))


def test_device_tensors_async(engine):
    import torch

    prof, dm = lyon_batch(4096, 128, 128, seed=5)
    tp = torch.from_numpy(prof).cuda()
    td = torch.from_numpy(dm).cuda()
    out = engine.lyon8(tp, td)
    engine.synchronize()
    check(out.cpu().numpy(), lyon8_batched(prof, dm))


def test_f64_rows_vs_oracle(engine):
    prof, dm = lyon_batch(300, 128, 200, seed=9)
    p = prof.astype(np.float64) / 3.0
    d = dm.astype(np.float64) * 1.7 - 20.0
    got = engine.lyon8(p, d)
    ref = lyon8_batched(p, d)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    m = ~np.isnan(ref)
    assert (np.abs(got - ref)[m] / np.maximum(1, np.abs(ref[m]))).max() <= 1e-12


def test_large_batch_properties(engine):
    """Full-size property check on device: 2M rows, mean bounds and repeatability."""
    import torch
    from pulsarfeatureextractor_amd.synth import lyon_batch_torch

    tp, td = lyon_batch_torch(2_000_000, 128, 128, seed=123)
    a = engine.lyon8(tp, td)
    b = engine.lyon8(tp, td)
    engine.synchronize()
    assert torch.equal(torch.nan_to_num(a), torch.nan_to_num(b)), "not deterministic"
    # exact mean from a torch integer reduction
    pm = tp.to(torch.int64).sum(dim=1).to(torch.float64) / 128.0
    assert torch.equal(a[:, 0], pm)
    # spot-check a random subset against the oracle
    idx = torch.randint(0, tp.shape[0], (2000,), generator=torch.Generator().manual_seed(0))
    sp, sd = tp[idx].cpu().numpy(), td[idx].cpu().numpy()
    check(a[idx].cpu().numpy(), lyon8_batched(sp, sd))


def test_config2_full_size_10m(engine):
    """BASELINE config 2 at the size it names, on the benched rows themselves (bench.py's
    generator and seed): one pfe_lyon8_u8 launch over 10M resident 128 + 128-byte candidates.
      * mean and std of both rows (columns 0, 1, 4, 5) bit-exact on EVERY row: numpy's sums
        of byte rows of 128 are exact, so x.sum() / 128 and sqrt(sum((x - mean)^2) / 128) are
        correctly rounded functions of the exact sums -- computed here with torch in fp64;
      * all 8 features of 2000 rows drawn from the last million against the oracle;
      * a 16384-row block tiled to 10M rows (as bench.py's config-3 line tiles): every tile
        bit-identical to the first (a grid-stride or 32-bit indexing fault past a few million
        rows breaks that)."""
    import torch
    from pulsarfeatureextractor_amd.synth import lyon_batch_torch

    n = 10_000_000
    tp, td = lyon_batch_torch(n, 128, 128, seed=20261017)   # bench.py's config-2 rows
    out = engine.lyon8(tp, td)
    engine.synchronize()
    for rows, (cm, cs) in ((tp, (0, 1)), (td, (4, 5))):
        for s in range(0, n, 1 << 20):
            x = rows[s:s + (1 << 20)].to(torch.float64)
            mean = x.sum(dim=1) / 128.0
            std = torch.sqrt(((x - mean[:, None]) ** 2).sum(dim=1) / 128.0)
            o = out[s:s + (1 << 20)]
            assert torch.equal(o[:, cm], mean), f"mean, rows {s}.."
            assert torch.equal(o[:, cs], std), f"std, rows {s}.."
    idx = torch.randint(n - 1_000_000, n, (2000,), generator=torch.Generator().manual_seed(7))
    check(out[idx].cpu().numpy(), lyon8_batched(tp[idx].cpu().numpy(), td[idx].cpu().numpy()))
    del out, tp, td
    blk = 16384
    bp, bd = lyon_batch_torch(blk, 128, 128, seed=20261018)
    reps = (n + blk - 1) // blk
    tp = bp.repeat(reps, 1)[:n].contiguous()
    td = bd.repeat(reps, 1)[:n].contiguous()
    out = engine.lyon8(tp, td)
    engine.synchronize()
    ob = out.view(torch.int64)
    full = (n // blk) * blk
    tiles = ob[:full].view(-1, blk, 8)
    bad = (tiles != tiles[:1]).any(dim=2).any(dim=1)
    assert not bool(bad.any()), f"tiles differing from tile 0: {torch.nonzero(bad)[:10].flatten().tolist()}"
    assert torch.equal(ob[full:], ob[: n - full])
    check(out[:blk].cpu().numpy(), lyon8_batched(bp.cpu().numpy(), bd.cpu().numpy()))
    del out, ob, tiles, tp, td
    torch.cuda.empty_cache()


def test_phcx_ndm120_full_size_1m(engine):
    """The benched real-PHCX shape at the size bench.py times (extra.lyon8_phcx_ndm120): one
    lyon8_u8_dm launch over 1M resident candidates of a 128-byte profile and a 120 x 128-byte
    DataBlock row (15 360 bytes), on bench.py's rows themselves (generator and seed):
      * the profile's mean and std and the DataBlock row's mean bit-exact on EVERY row (byte
        sums are exact, so numpy's x.sum() / L is the correctly rounded quotient; the 128-byte
        profile's centred squares sum exactly as well) -- computed here with torch in fp64;
      * all 8 features of 600 rows drawn from the last 100k against the oracle, mean/std of
        both rows bit-exact (the DataBlock std follows numpy's 8192-element chunks);
      * a 4096-row block tiled to 1M rows: every tile bit-identical to the first, the first
        200 rows against the oracle (a grid-stride or 32-bit offset fault past 2^31 bytes of
        DataBlock rows -- 140k rows -- breaks that)."""
    import torch
    from pulsarfeatureextractor_amd.synth import lyon_batch_torch

    n, ld = 1_000_000, 15360
    tp, td = lyon_batch_torch(n, 128, ld, seed=20261023)   # bench.py run_lyon8_phcx(ld=15360)
    out = engine.lyon8(tp, td)
    engine.synchronize()
    for s in range(0, n, 1 << 17):
        x = tp[s:s + (1 << 17)].to(torch.float64)
        mean = x.sum(dim=1) / 128.0
        std = torch.sqrt(((x - mean[:, None]) ** 2).sum(dim=1) / 128.0)
        # numpy's x.sum() / ld: an exact integer sum divided once, correctly rounded (on the
        # host: torch divides by a scalar through its reciprocal)
        d = torch.from_numpy(td[s:s + (1 << 17)].to(torch.float64).sum(dim=1).cpu().numpy()
                             / float(ld)).to(out.device)
        o = out[s:s + (1 << 17)]
        assert torch.equal(o[:, 0], mean), f"profile mean, rows {s}.."
        assert torch.equal(o[:, 1], std), f"profile std, rows {s}.."
        assert torch.equal(o[:, 4], d), f"DataBlock mean, rows {s}.."
    idx = torch.randint(n - 100_000, n, (600,), generator=torch.Generator().manual_seed(11))
    check(out[idx].cpu().numpy(), lyon8_batched(tp[idx].cpu().numpy(), td[idx].cpu().numpy()))
    del out, tp, td
    torch.cuda.empty_cache()
    blk = 4096
    bp, bd = lyon_batch_torch(blk, 128, ld, seed=20261024)
    reps = (n + blk - 1) // blk
    tp = bp.repeat(reps, 1)[:n].contiguous()
    td = bd.repeat(reps, 1)[:n].contiguous()
    out = engine.lyon8(tp, td)
    engine.synchronize()
    ob = out.view(torch.int64)
    full = (n // blk) * blk
    tiles = ob[:full].view(-1, blk, 8)
    bad = (tiles != tiles[:1]).any(dim=2).any(dim=1)
    assert not bool(bad.any()), f"tiles differing from tile 0: {torch.nonzero(bad)[:10].flatten().tolist()}"
    assert torch.equal(ob[full:], ob[: n - full])
    check(out[:200].cpu().numpy(), lyon8_batched(bp[:200].cpu().numpy(), bd[:200].cpu().numpy()))
    del out, ob, tiles, tp, td
    torch.cuda.empty_cache()


@pytest.mark.parametrize("lp,ld", [(128, 15360), (128, 16384), (64, 7680), (256, 8192),
                                   (128, 12800), (128, 8320), (64, 384), (256, 10240),
                                   (64, 16384), (256, 16384), (128, 8192), (64, 8192),
                                   (64, 14336), (256, 13312), (128, 12288)])
def test_long_dm_rows_vs_oracle(engine, lp, ld):
    """The real PHCX shape: a 64-256-bin profile and the whole section-0 DataBlock (nDM x
    128 bytes; nDM = 120, 128, 60, 64, 100, 65, 3, 80, 112, 104, 96).  Kernels: nDM = 64 / 128
    lyon8_u8_pow2 (exact leaf sums); every other length here lyon8_u8_dm (one wave per row,
    numpy's chains byte by byte).  mean and std bit-exact for both rows -- the DM row's std
    follows numpy's own reduction (8192-element chunks, each a pairwise tree) -- skew/kurt
    within 1e-12."""
    prof, dm = lyon_batch(300, lp, ld, seed=31 + ld, adversarial=True)
    got = engine.lyon8(prof, dm)
    check(got, lyon8_batched(prof, dm), exact_cols=(0, 1, 4, 5))


@pytest.mark.parametrize("ld", [15360, 12800, 9216, 16256, 30720])
def test_long_dm_rows_multibatch(engine, ld):
    """lyon8_u8_dm with one block (4 waves) over 600 rows: every wave runs several batches of
    up to 64 rows (finalised one row per lane), the last one partial.  Bit-identical to the
    default grid, mean/std bit-exact against the oracle."""
    prof, dm = lyon_batch(600, 128, ld, seed=3 + ld, adversarial=True)
    ref = engine.lyon8(prof, dm)
    with engine.options(lyon8_blocks=1):
        got = engine.lyon8(prof, dm)
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))
    check(got, lyon8_batched(prof, dm), exact_cols=(0, 1, 4, 5))


@pytest.mark.parametrize("opt", [1, 2])
def test_long_dm_rows_kernel_options_agree(engine, opt):
    """The other DataBlock kernel options (PFE_OPT_LYON8_DM: 1 the round-3 kernels, 2 the
    exact integer power sums instead of the default's fp64 moments) against the default: the
    same mean/std bits; skew/kurt agree to 1e-12, and each is held to the oracle like the
    default."""
    prof, dm = lyon_batch(400, 128, 15360, seed=77, adversarial=True)
    a = engine.lyon8(prof, dm)
    with engine.options(lyon8_dm=opt):
        b = engine.lyon8(prof, dm)
    for c in (0, 1, 4, 5):
        assert np.array_equal(a[:, c], b[:, c], equal_nan=True)
    m = ~np.isnan(b)
    assert np.array_equal(np.isnan(a), np.isnan(b))
    assert (np.abs(a - b)[m] / np.maximum(1, np.abs(b[m]))).max() <= TOL
    check(b, lyon8_batched(prof, dm), exact_cols=(0, 1, 4, 5))


@pytest.mark.parametrize("ld", [16256, 4352, 30720, 24576, 6272])
def test_long_dm_rows_other_lengths(engine, ld):
    """DataBlock lengths outside the round-3 fast set, all through lyon8_u8_dm (round 4):
    nDM = 127 / 34 / 49 (the last chunk's leaves differ in length -- 120 and 128, 64 and 72,
    96 and 104 -- on a perfect tree), 240 / 192 (four and three numpy chunks) -- mean and std
    bit-exact, skew/kurt within 1e-12."""
    prof, dm = lyon_batch(200, 128, ld, seed=7 + ld, adversarial=True)
    got = engine.lyon8(prof, dm)
    check(got, lyon8_batched(prof, dm), exact_cols=(0, 1, 4, 5))


@pytest.mark.parametrize("lp,ld", [(128, 4224), (128, 12416), (128, 20608), (128, 28800),
                                   (64, 12416), (256, 4224)])
def test_long_dm_rows_imperfect_trees(engine, lp, ld):
    """nDM = 33 / 97 / 161 / 225: the DataBlock lengths <= 256 rows whose last numpy chunk
    (4224 bytes) is not a perfect tree -- 16 blocks of 128 + (64 + 72), leaves at two
    depths -- through lyon8_u8_dm's tri form (round 5): mean and std bit-exact like every
    other length, skew / kurt within 1e-12."""
    prof, dm = lyon_batch(300, lp, ld, seed=9 + ld + lp, adversarial=True)
    got = engine.lyon8(prof, dm)
    check(got, lyon8_batched(prof, dm), exact_cols=(0, 1, 4, 5))


def test_long_dm_rows_golden_dmplane(engine):
    """Against the reference's own outputs for 128-bin PHCX files whose section-0 DataBlock
    is a 120 x 128 period-DM plane (tests/golden/lyon8_phcx128_dmplane.npz)."""
    from golden_util import load

    d = load("lyon8_phcx128_dmplane")
    prof = np.ascontiguousarray(d["prof"], dtype=np.uint8)
    dm = np.ascontiguousarray(d["block0"], dtype=np.uint8)
    got = engine.lyon8(prof, dm)
    ok = d["ok"].astype(bool)
    check(got[ok], d["out"][ok], exact_cols=(0, 1, 4, 5))


@pytest.mark.parametrize("lp,ld", [(128, 3840), (128, 9216), (128, 20480), (64, 1024),
                                   (128, 8448), (256, 10240), (128, 2048), (128, 24704),
                                   (128, 4224), (128, 12416), (64, 28800), (64, 4224),
                                   (256, 4224)])
def test_long_dm_rows_split_last_chunk(engine, lp, ld):
    """Last numpy chunks of <= 32 leaves (nDM = 30, 72, 160, 8, 66, 80, 16, 193: 32, 8, 32, 8,
    2, 16, 16 and 1 leaves) summed by 2, 4 or 8 lanes per leaf, each with some of the leaf's 8
    chains, the tri form (nDM = 33, 97, 225) with its 128-byte leaves split over the quad's
    idle lane, and one-chunk rows of <= 32 leaves (nDM = 30, 8, 16) two per wave (round 5,
    PFE_OPT_LYON8_DM_SPLIT 1; 2 = the chain splits only), and since round 6 the one-chunk tri
    rows (nDM = 33, 64/128/256-byte profiles) two per wave as well, two lanes per 264-byte
    block (G = 32; option 2 keeps the quad split): mean and std bit-identical to one
    lane per leaf and bit-exact against the oracle; skew / kurt (their d^3 / d^4 sums are
    grouped by lane, in any order) within 1e-12 of one lane per leaf.  An odd row count and a
    one-block grid (several 64-row batches per wave, a lone last row) cover the pairs' edges."""
    prof, dm = lyon_batch(301, lp, ld, seed=5 + ld + lp, adversarial=True)
    with engine.options(lyon8_dm_split=0):
        one = engine.lyon8(prof, dm)
    ref = lyon8_batched(prof, dm)
    for opts in ({}, {"lyon8_dm_split": 2}, {"lyon8_blocks": 1}):
        with engine.options(**opts):
            got = engine.lyon8(prof, dm)
        for c in (0, 1, 4, 5):
            assert np.array_equal(got[:, c].view(np.uint64), one[:, c].view(np.uint64)), (opts, c)
        m = ~np.isnan(one)
        assert np.array_equal(np.isnan(got), np.isnan(one))
        assert (np.abs(got - one)[m] / np.maximum(1, np.abs(one[m]))).max() <= TOL
        check(got, ref, exact_cols=(0, 1, 4, 5))
