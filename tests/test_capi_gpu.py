"""The C-ABI's host-facing behaviour on the GPU: handle options, argument checks of the
device path (nothing mis-typed reaches a kernel), cross-stream ordering of one handle, and
the chunked, pipelined host-pointer path (pinned and pageable buffers)."""
import numpy as np
import pytest

from pulsarfeatureextractor_amd._native import Engine, PfeError, host_empty
from pulsarfeatureextractor_amd.synth import bates_batch, lyon_batch

pytestmark = pytest.mark.gpu


def test_options_roundtrip_and_range(engine):
    assert engine.get_option("solver") == 0
    assert engine.get_option("lyon8_burst") == 2
    with engine.options(solver="batched", gslots=5, lyon8_burst=4):
        assert engine.get_option("solver") == 1
        assert engine.get_option("gslots") == 5
    assert engine.get_option("solver") == 0 and engine.get_option("gslots") == 0
    for name, bad in (("solver", 3), ("serial", 2), ("gslots", 33), ("lyon8_burst", 3),
                      ("pfd_waves", 2), ("lyon8_blocks", 0)):
        with pytest.raises(PfeError):
            engine.set_option(name, bad)


def test_lyon8_burst_and_grid_options_same_bits(engine):
    prof, dm = lyon_batch(5000, 128, 128, seed=3)
    ref = engine.lyon8(prof, dm)
    for kw in ({"lyon8_burst": 1}, {"lyon8_burst": 4}, {"lyon8_blocks": 7}):
        with engine.options(**kw):
            got = engine.lyon8(prof, dm)
        assert np.array_equal(np.nan_to_num(got, nan=7.0), np.nan_to_num(ref, nan=7.0)), kw


def test_device_arguments_are_checked(engine):
    import torch

    b = bates_batch(32, seed=2)
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in b.items()}
    with pytest.raises(TypeError):   # float32 DM curve: would be read as n*ndm*8 bytes
        engine.bates22(t["prof"], t["sub"], t["dmcurve"].float(), t["scal"])
    with pytest.raises(TypeError):   # integer profile reinterpreted as bytes
        engine.bates22(t["prof"].int(), t["sub"], t["dmcurve"], t["scal"])
    with pytest.raises(ValueError):  # short output
        engine.bates22(t["prof"], t["sub"], t["dmcurve"], t["scal"],
                       out=torch.empty((31, 22), dtype=torch.float64, device="cuda"))
    with pytest.raises(ValueError):  # status of the wrong length
        engine.bates22(t["prof"], t["sub"], t["dmcurve"], t["scal"],
                       status=torch.empty((16,), dtype=torch.int32, device="cuda"))
    with pytest.raises(TypeError):   # status of the wrong width
        engine.bates22(t["prof"], t["sub"], t["dmcurve"], t["scal"],
                       status=torch.empty((32,), dtype=torch.int64, device="cuda"))
    with pytest.raises(ValueError):  # non-contiguous
        engine.subband3(t["prof"], t["sub"].transpose(1, 2), t["scal"])
    with pytest.raises(TypeError):   # mixed host / device
        engine.bates22(t["prof"], b["sub"], t["dmcurve"], t["scal"])
    p, d = lyon_batch(16, 64, 64)
    tp = torch.from_numpy(p).cuda()
    with pytest.raises(TypeError):
        engine.lyon8(tp, torch.from_numpy(d).cuda().to(torch.float64))


def test_two_streams_one_handle_are_ordered():
    """One handle used under two torch streams: the second call waits for the first (the
    shared workspace and work queues are never used by two chains at once)."""
    import torch

    b = bates_batch(400, seed=12)
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in b.items()}
    with Engine(0) as e:
        ref, rst = e.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        outs = []
        for s in (s1, s2, s1, s2):
            with torch.cuda.stream(s):
                outs.append(e.bates22(t["prof"], t["sub"], t["dmcurve"], t["scal"]))
        torch.cuda.synchronize()
    for o, st in outs:
        assert np.array_equal(st.cpu().numpy().view(np.uint32), rst)
        assert np.array_equal(np.nan_to_num(o.cpu().numpy(), nan=7.0), np.nan_to_num(ref, nan=7.0))


@pytest.mark.parametrize("pinned", [False, True])
def test_chunked_host_path(engine, pinned):
    """n spanning several pipeline chunks (131072 rows of 256 B each): host staging and the
    pinned in-place DMA give the device path's bits, strided rows included."""
    import torch

    n = 300_001
    prof, dm = lyon_batch(n, 128, 128, seed=77)
    if pinned:
        hp, hd = host_empty(prof.shape, np.uint8), host_empty(dm.shape, np.uint8)
        hp[:] = prof
        hd[:] = dm
        out = host_empty((n, 8), np.float64)
    else:
        hp, hd, out = prof, dm, None
    got = engine.lyon8(hp, hd, out=out)
    ref = engine.lyon8(torch.from_numpy(prof).cuda(), torch.from_numpy(dm).cuda())
    engine.synchronize()
    ref = ref.cpu().numpy()
    assert np.array_equal(np.nan_to_num(got, nan=7.0), np.nan_to_num(ref, nan=7.0))
    # strided rows (every other row of a wider array)
    wide = np.zeros((2 * 5000, 160), dtype=np.uint8)
    wide[::2, :128] = prof[:5000]
    got2 = engine.lyon8(wide[::2, :128], dm[:5000])
    assert np.array_equal(np.nan_to_num(got2, nan=7.0), np.nan_to_num(ref[:5000], nan=7.0))
