"""Config 5 on the GPU: the (n, 30) feature matrix (8 Lyon features + 22 Bates scores of each
candidate) against the reference's own 30 values of the same files (tests/golden/
all30_phcx128.npz, tools/make_golden.py mode "all30"), and the multi-rank path
(distributed.score_sharded) around the real Engine: two ranks started with spawn, sharing
cuda:0, gathering over gloo, must reproduce the single-process matrix bit for bit; and one
rank in an RCCL ("nccl") group of one, gathering device tensors with all_gather_into_tensor,
so the collective the 8-GPU run uses has run on this GPU."""
import json
import os
import socket

import numpy as np
import pytest

from golden_util import GOLDEN, bates_inputs, load
from golden_util import envelope_check
from test_bates22_gpu import BITEXACT, check_against

pytestmark = pytest.mark.gpu


def all30_inputs(d):
    prof, sub, curve, scal = bates_inputs(d)
    return prof, d["block0"], sub, curve, scal


def test_features30_vs_reference_golden(engine):
    d = load("all30_phcx128")
    prof, lyon_dm, sub, curve, scal = all30_inputs(d)
    out, st = engine.features30(prof, lyon_dm, sub, curve, scal)
    ok = d["ok"]
    ref = d["out"]
    # the 8 Lyon features: mean/std bit-exact, skew/kurt within 1e-12 (tests/test_lyon8_gpu.py)
    l8 = out[:, :8]
    with np.errstate(all="ignore"):
        r = np.abs(l8[ok] - ref[ok][:, :8]) / np.maximum(1.0, np.abs(ref[ok][:, :8]))
    assert np.array_equal(l8[ok][:, [0, 1, 4, 5]], ref[ok][:, [0, 1, 4, 5]])
    assert np.nanmax(r) <= 1e-12
    # the 22 scores under the 22-score bar (population floor of the PHCX golden set)
    floor = json.load(open(os.path.join(GOLDEN, "chaos_floor.json")))["bates22_phcx128"]
    rmax = np.load(os.path.join(GOLDEN, "chaos_rows.npz"))["all30_phcx128_rmax"]
    check_against(out[:, 8:], st, np.where(ok[:, None], ref[:, 8:], np.nan), ok, "all30", floor,
                  rmax=rmax)
    envelope_check(out[:, 8:], st, "all30_phcx128", skip=BITEXACT, cols=slice(8, None))


def test_features30_device_matches_host(engine):
    import torch

    d = load("all30_phcx128")
    arrs = all30_inputs(d)
    host, hst = engine.features30(*arrs)
    t = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]
    dev, dst = engine.features30(*t)
    engine.synchronize()
    assert np.array_equal(np.nan_to_num(dev.cpu().numpy(), nan=7.0), np.nan_to_num(host, nan=7.0))
    assert np.array_equal(dst.cpu().numpy().view(np.uint32), hst)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist

    from pulsarfeatureextractor_amd import distributed as D
    from pulsarfeatureextractor_amd._native import Engine

    D.init_from_env("gloo")
    d = load("all30_phcx128")
    arrs = dict(zip(("prof", "lyon_dm", "sub", "dmcurve", "scal"), all30_inputs(d)))
    n = len(arrs["prof"])
    with Engine(0) as eng:
        def score(prof, lyon_dm, sub, dmcurve, scal):
            out, st = eng.features30(prof, lyon_dm, sub, dmcurve, scal)
            return torch.from_numpy(np.concatenate([out, st.astype(np.float64)[:, None]], axis=1))

        full = D.score_sharded(score, arrs, n)
    q.put((rank, full.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_score_sharded_with_engine(engine):
    import torch.multiprocessing as mp

    d = load("all30_phcx128")
    arrs = all30_inputs(d)
    out, st = engine.features30(*arrs)
    single = np.concatenate([out, st.astype(np.float64)[:, None]], axis=1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in (0, 1):
        assert res[r].shape == single.shape
        assert np.array_equal(np.nan_to_num(res[r], nan=7.0), np.nan_to_num(single, nan=7.0)), r


def _rank_rccl1(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    import torch
    import torch.distributed as dist

    from pulsarfeatureextractor_amd import distributed as D
    from pulsarfeatureextractor_amd._native import Engine

    rank, world = D.init_from_env("nccl", group_at_one=True)
    assert dist.is_initialized() and dist.get_backend() == "nccl" and world == 1
    d = load("all30_phcx128")
    arrs = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda()
            for k, v in zip(("prof", "lyon_dm", "sub", "dmcurve", "scal"), all30_inputs(d))}
    n = int(arrs["prof"].shape[0])
    with Engine(0) as eng:
        def score(prof, lyon_dm, sub, dmcurve, scal):
            out, st = eng.features30(prof, lyon_dm, sub, dmcurve, scal)
            eng.synchronize()
            return torch.cat([out, st.to(torch.float64)[:, None]], dim=1)

        full = D.score_sharded(score, arrs, n)          # RCCL all_gather_into_tensor
        local = score(**arrs)
        # an uneven shard layout through the padded path: 3 of the rows as "this rank's"
        part = D.gather_rows(local[:3].contiguous(), 3)
    torch.cuda.synchronize()
    res = (full.device.type, full.cpu().numpy(), local.cpu().numpy(), part.cpu().numpy())
    q.put(res)
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_group_of_one_gathers_device_matrix(engine):
    """SURVEY.md 8(e) / north_star's RCCL all-gather: init_from_env("nccl") with WORLD_SIZE = 1
    and score_sharded / gather_rows over device tensors of the (n, 30) matrix."""
    import torch.multiprocessing as mp

    d = load("all30_phcx128")
    out, st = engine.features30(*all30_inputs(d))
    single = np.concatenate([out, st.astype(np.float64)[:, None]], axis=1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rank_rccl1, args=(_free_port(), q))
    p.start()
    dev, full, local, part = q.get(timeout=240)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert dev == "cuda"
    same = lambda a, b: np.array_equal(np.nan_to_num(a, nan=7.0), np.nan_to_num(b, nan=7.0))
    assert same(full, single) and same(local, single) and same(part, single[:3])
