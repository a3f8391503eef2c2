"""Candidate-parallel execution across the GPUs of a node.

Candidates are independent, so each rank scores a contiguous shard
[r*N/W, (r+1)*N/W) with no communication.  The only collective is the optional
reassembly of the feature matrix: an all-gather (RCCL over xGMI with backend "nccl", gloo
on CPU) of equal-size padded shards, trimmed back to N rows on every rank.

One process per GPU (torchrun / torch.distributed.run); rank r uses cuda:LOCAL_RANK.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous shard of rank `rank`: rows [lo, hi)."""
    return (n * rank) // world, (n * (rank + 1)) // world


def init_from_env(backend: str | None = None, group_at_one: bool = False):
    """Initialise the default process group from RANK/WORLD_SIZE/MASTER_* (127.0.0.1).
    With WORLD_SIZE = 1 no group is made unless `group_at_one` (a one-rank RCCL group, so
    the collective path can run on a single GPU)."""
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world == 1 and not group_at_one:
        return 0, 1
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl":
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        kw["device_id"] = torch.device("cuda", local)
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return rank, world


def gather_rows(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather the row shards of every rank (shard_bounds layout) -> (n_total, F).

    Shards differ by at most one row; each is padded to the largest before the
    all_gather_into_tensor so the collective moves one contiguous buffer per rank."""
    world = dist.get_world_size(group)
    rows = [shard_bounds(n_total, world, r) for r in range(world)]
    width = max(hi - lo for lo, hi in rows)
    equal = all(hi - lo == width for lo, hi in rows)
    if equal and local.is_contiguous():
        pad = local  # equal shards (n_total divisible by world): no padding, no trimming copy
    else:
        pad = torch.zeros((width,) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
        pad[: local.shape[0]] = local
    buf = torch.empty((world * width,) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    dist.all_gather_into_tensor(buf, pad, group=group)
    if equal:
        return buf
    parts = [buf[r * width: r * width + (hi - lo)] for r, (lo, hi) in enumerate(rows)]
    return torch.cat(parts, dim=0)


def score_sharded(score_fn, arrays: dict, n_total: int, gather: bool = True, group=None):
    """Run `score_fn(**shard_arrays) -> tensor (rows, F)` on this rank's shard of every
    array in `arrays` (row-sliced), then optionally all-gather the result."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    lo, hi = shard_bounds(n_total, world, rank)
    local = score_fn(**{k: v[lo:hi] for k, v in arrays.items()})
    if not gather or not dist.is_initialized():
        return local
    return gather_rows(local, n_total, group)
