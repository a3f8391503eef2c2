"""world_size-2 gloo run of the candidate-sharded path (no GPU): each rank scores its
contiguous shard with the oracle standing in for the kernel (tests may use the oracle as
the checker), the all-gather reassembles the matrix, and the result equals the single-
process result row for row."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from pulsarfeatureextractor_amd.distributed import shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch.distributed as dist

    from oracle.lyon import lyon8_batched
    from pulsarfeatureextractor_amd import distributed as D
    from pulsarfeatureextractor_amd.synth import lyon_batch

    D.init_from_env("gloo")
    prof, dm = lyon_batch(n, 64, 64, seed=3)

    def fn(prof, dm):
        return torch.from_numpy(lyon8_batched(prof, dm))

    full = D.score_sharded(fn, {"prof": prof, "dm": dm}, n)
    q.put((rank, full.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [1001, 8])
def test_gloo_world2_matches_single(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle.lyon import lyon8_batched
    from pulsarfeatureextractor_amd.synth import lyon_batch

    prof, dm = lyon_batch(n, 64, 64, seed=3)
    ref = lyon8_batched(prof, dm)
    for r in (0, 1):
        assert np.array_equal(np.nan_to_num(res[r], nan=9.0), np.nan_to_num(ref, nan=9.0))


def test_shard_bounds_partition():
    for n in (0, 1, 7, 10_000_001):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1
