"""ORACLE (test infrastructure only) — the 22-score restatement (oracle.bates) spread over host
processes, for bench.py's multi-core CPU baseline (the reference-equivalent
loop on all host cores via multiprocessing).  libpfe.so never calls it.

Workers are started with the "spawn" method (a fresh interpreter per worker, no state copied
from a parent that may hold a GPU context) with one BLAS/OpenMP thread each.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import time
import warnings


def _chunk(args):
    prof, sub, curve, scal = args
    from oracle.bates import bates22

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        t0 = time.perf_counter()
        bates22(prof, sub, curve, scal)
        return time.perf_counter() - t0


def bates22_multicore(prof, sub, curve, scal, workers):
    """Score the rows on `workers` processes (contiguous chunks); returns the wall seconds of
    the scoring map, the pool already started and warmed (one tiny chunk per worker)."""
    saved = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    for k in saved:
        os.environ[k] = "1"
    try:
        ctx = mp.get_context("spawn")
        with ctx.Pool(workers) as pool:
            warm = [(prof[:2], sub[:2], curve[:2], scal[:2])] * workers
            pool.map(_chunk, warm, chunksize=1)
            n = len(prof)
            cuts = [n * i // workers for i in range(workers + 1)]
            parts = [(prof[a:b], sub[a:b], curve[a:b], scal[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
            t0 = time.perf_counter()
            pool.map(_chunk, parts, chunksize=1)
            return time.perf_counter() - t0
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
