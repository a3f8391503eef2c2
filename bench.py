#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X feature engine.

metric (BASELINE.json): candidates/sec of the 8-feature (Lyon) path on synthetic 128-bin
profile + 128-bin DM rows, plus HBM GB/s vs peak.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--n ROWS_PER_GPU]
                  [--path lyon8|bates22|pfd|pfd22]

One "step" = one pass of the hot path (pfe_lyon8_u8 through the C-ABI, device pointers,
inputs resident in HBM) over the rank's whole batch of synthetic candidates (config 2:
10M rows per GPU).  For N > 1 the driver starts one process per GPU with
torch.distributed.run; candidates shard with no data-path collective (weak scaling:
10M rows per rank); the timed region is bracketed by barrier + synchronize and the MAX over
ranks is reported; value = all rows processed by all ranks / that time.

Besides the contract fields the JSON line carries:
  roofline     : the lyon8 kernel's algorithmic bytes per launch (n * (lp + ld + 64) B)
                 / its average duration, measured with HIP events on the stream the kernel
                 runs on, against the 8.0 TB/s HBM3E peak; traffic = PMC-measured HBM bytes
                 per launch from profiles/ when a matching summary is committed, else null
  cpu_baseline : the reference-equivalent per-candidate numpy/scipy loop (oracle.lyon.lyon8,
                 the scalar port of PHCXFile.py:320-379) timed on this host, 1 core, on a
                 bounded sample of the same synthetic rows (rank 0, N=1 only)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=None,
                    help="candidates per GPU (default 10M for lyon8, 1M for bates22)")
    ap.add_argument("--lp", type=int, default=128)
    ap.add_argument("--ld", type=int, default=128)
    ap.add_argument("--path", choices=["lyon8", "bates22", "all30", "pfd", "pfd22"], default="lyon8",
                    help="all30: config 5's 8 Lyon features + 22 Bates scores per candidate "
                         "into one (n, 30) feature matrix")
    ap.add_argument("--pfd-shape", default="16x32x128", help="npart x nsub x proflen (pfd path)")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="rows for the CPU baseline sample (default 8000 lyon8 / 300 bates22; 0 disables)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cpu-multicore", action="store_true",
                    help="skip the multi-process CPU baseline of the 22-score paths")
    ap.add_argument("--gather", action="store_true",
                    help="also time the RCCL all-gather that reassembles the feature matrix")
    return ap.parse_args()


def load_traffic(name: str):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (profiles/*.json)."""
    p = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_baseline_lyon8(lp, ld, sample):
    import numpy as np

    from oracle.lyon import lyon8
    from pulsarfeatureextractor_amd.synth import lyon_batch

    prof, dm = lyon_batch(sample, lp, ld, seed=4242)
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        lyon8(prof[:50], dm[:50])  # warm imports
        t0 = time.perf_counter()
        lyon8(prof, dm)
        dt = time.perf_counter() - t0
    return {
        "value": sample / dt,
        "unit": "candidates/sec",
        "cores": 1,
        "kind": "port",
        "sample": f"{sample} synthetic {lp}-bin profile + {ld}-bin DM rows through the "
                  f"reference-equivalent per-candidate numpy.mean/std + scipy.stats.skew/"
                  f"kurtosis loop (oracle.lyon.lyon8), {dt:.1f} s on 1 host core",
    }


def cpu_baseline_lyon8_omp(lp, ld, sample=2_000_000):
    """the C restatement (oracle/c/lyon8_omp.c) with OpenMP on the host
    cores this job has (OMP_NUM_THREADS, 16 on the GPU box); None when it is not built."""
    from oracle import lyon_c
    from pulsarfeatureextractor_amd.synth import lyon_batch

    if not lyon_c.available():
        return None
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    prof, dm = lyon_batch(sample, lp, ld, seed=4244)
    lyon_c.lyon8_omp(prof[:10000], dm[:10000], threads)  # warm the thread pool
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        lyon_c.lyon8_omp(prof, dm, threads)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return {
        "value": sample / best,
        "unit": "candidates/sec",
        "cores": threads,
        "kind": "port",
        "sample": f"{sample} synthetic {lp}-bin profile + {ld}-bin DM rows through the C "
                  f"restatement (oracle/c/lyon8_omp.c, two-pass float64 moments), best of 3, "
                  f"{best * 1e3:.0f} ms on {threads} OpenMP threads",
    }


def cpu_baseline_bates22(lp, sample):
    import warnings

    from oracle.bates import bates22
    from pulsarfeatureextractor_amd.synth import bates_batch

    b = bates_batch(sample, lp=lp, lsb=lp, seed=4243)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        bates22(b["prof"][:5], b["sub"][:5], b["dmcurve"][:5], b["scal"][:5])
        t0 = time.perf_counter()
        bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
        dt = time.perf_counter() - t0
    return {
        "value": sample / dt,
        "unit": "candidates/sec",
        "cores": 1,
        "kind": "port",
        "sample": f"{sample} synthetic config-3 candidates ({lp}-bin profile, 16x{lp} sub-bands, "
                  f"128-point DM curve) through the reference-equivalent numpy/scipy.optimize."
                  f"leastsq restatement (oracle.bates.bates22), {dt:.1f} s on 1 host core",
    }


def cpu_baseline_bates22_mp(lp, per_worker=300):
    """SURVEY.md §8(d)(i) on all host cores: the same restatement in `workers` spawned
    processes (16 on the GPU box's CPU share), per_worker candidates each."""
    from oracle.bates_mp import bates22_multicore
    from pulsarfeatureextractor_amd.synth import bates_batch

    workers = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    n = workers * per_worker
    b = bates_batch(n, lp=lp, lsb=lp, seed=4245)
    dt = bates22_multicore(b["prof"], b["sub"], b["dmcurve"], b["scal"], workers)
    return {
        "value": n / dt,
        "unit": "candidates/sec",
        "cores": workers,
        "kind": "port",
        "sample": f"{n} synthetic config-3 candidates through oracle.bates.bates22 in {workers} "
                  f"spawned processes (one BLAS thread each), {dt:.1f} s wall",
    }


def pfd_block(n, shape, seed):
    """n synthetic PRESTO folds of one shape -> pfe_pfd_dmprof inputs (numpy)."""
    import numpy as np

    from pulsarfeatureextractor_amd import pfd as _pfd
    from pulsarfeatureextractor_amd.synth import pfd_candidate

    npart, nsub, L = shape
    datas = []
    for i in range(n):
        c = pfd_candidate(np.random.default_rng(seed + i), npart, nsub, L)
        chanpersub = c["numchan"] // nsub
        sd = c["chan_wid"] * chanpersub
        stats = c["stats"]
        datas.append(_pfd.PFDData(
            npart=npart, nsub=nsub, proflen=L, profs=c["profs"], bestdm=c["bestdm"],
            binspersec=c["fold_p1"] * L, avgprof=(c["profs"] / L).sum(),
            varprof=float(stats[:, :, 5].sum()), dms=c["dms"], numdms=len(c["dms"]),
            bary_p1=c["fold_p1"],
            subfreqs=np.arange(nsub, dtype="d") * sd + (c["lofreq"] + sd - c["chan_wid"])))
    return datas


def cpu_baseline_pfd(shape, sample):
    import warnings

    from oracle.pfd import lyon8_one

    datas = pfd_block(sample, shape, 4244)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        lyon8_one(datas[0])
        t0 = time.perf_counter()
        for d in datas:
            lyon8_one(d)
        dt = time.perf_counter() - t0
    return {
        "value": sample / dt, "unit": "candidates/sec", "cores": 1, "kind": "port",
        "sample": f"{sample} synthetic {shape[0]}x{shape[1]}x{shape[2]} PRESTO folds through "
                  f"the reference-equivalent numpy/scipy dedisperse + getprofile + "
                  f"plot_chi2_vs_DM + stats restatement (oracle.pfd.lyon8_one), {dt:.1f} s on "
                  f"1 host core",
    }


def cpu_baseline_pfd22(shape, sample):
    import warnings

    from oracle.bates import CandidateFailure
    from oracle.pfd import bates22_one

    datas = pfd_block(sample, shape, 4245)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        t0 = time.perf_counter()
        for d in datas:
            try:
                bates22_one(d)
            except CandidateFailure:
                pass
        dt = time.perf_counter() - t0
    return {
        "value": sample / dt, "unit": "candidates/sec", "cores": 1, "kind": "port",
        "sample": f"{sample} synthetic {shape[0]}x{shape[1]}x{shape[2]} PRESTO folds through "
                  f"the reference-equivalent numpy/scipy PFDFile.compute restatement "
                  f"(oracle.pfd.bates22_one), {dt:.1f} s on 1 host core",
    }


def load_ops_per_candidate():
    p = os.path.join(ROOT, "profiles", "r01_bates22_ops.json")
    try:
        with open(p) as f:
            return json.load(f)["ops_per_candidate"]
    except Exception:
        return None


def main():
    args = parse()
    if args.n is None:
        args.n = {"lyon8": 10_000_000, "bates22": 1_000_000, "all30": 1_000_000, "pfd": 32768,
                  "pfd22": 32768}[args.path]
    if args.cpu_sample is None:
        args.cpu_sample = {"lyon8": 8000, "bates22": 300, "all30": 300, "pfd": 200,
                           "pfd22": 60}[args.path]
    pfd_shape = tuple(int(v) for v in args.pfd_shape.split("x"))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    # PFE_BENCH_BACKEND=gloo (rehearsal only): N ranks sharing the GPUs there are, the
    # barrier / max-over-ranks reduction over gloo; the driver's runs use RCCL ("nccl")
    backend = os.environ.get("PFE_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist_on = world > 1
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    from pulsarfeatureextractor_amd._native import Engine
    from pulsarfeatureextractor_amd.synth import lyon_batch_torch

    eng = Engine(local)
    stream = torch.cuda.Stream(device=local)  # the kernel's stream; events record on it
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)

    n = args.n
    dev = f"cuda:{local}"
    if args.path == "lyon8":
        # rank-specific synthetic shard, resident in HBM before timing
        prof, dm = lyon_batch_torch(n, args.lp, args.ld, seed=20261017 + rank, device=dev)
        out = torch.empty((n, 8), dtype=torch.float64, device=dev)

        def step():
            eng.lyon8(prof, dm, out=out)
    elif args.path in ("pfd", "pfd22"):
        import numpy as np

        from pulsarfeatureextractor_amd import pfd as _pfd

        blk = 1024  # synthetic folds generated on the host, tiled to n rows in HBM
        profs, subfreqs, pscal = _pfd.batch_inputs(pfd_block(blk, pfd_shape, 20261019 + rank))
        reps = (n + blk - 1) // blk

        def tile(a):
            t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
            return t.repeat((reps,) + (1,) * (t.dim() - 1))[:n].contiguous()

        tp, tf, ts = tile(profs), tile(subfreqs), tile(pscal)
        del profs

        if args.path == "pfd":
            def step():
                eng.pfd_dmprof(tp, tf, ts, profile=False, chis=False, lyon8=True)
        else:
            out = torch.empty((n, 22), dtype=torch.float64, device=dev)
            status = torch.empty((n,), dtype=torch.int32, device=dev)

            def step():
                eng.pfd_bates22(tp, tf, ts, out=out, status=status)
    else:
        import numpy as np

        from pulsarfeatureextractor_amd.synth import bates_batch

        # a 16384-candidate synthetic block (SURVEY.md §8(d) recipe), tiled to n rows in HBM
        base = bates_batch(16384, lp=args.lp, lsb=args.lp, seed=20261018 + rank)
        reps = (n + 16383) // 16384
        bt = {}
        for k, v in base.items():
            t = torch.from_numpy(np.ascontiguousarray(v)).to(dev)
            bt[k] = t.repeat((reps,) + (1,) * (t.dim() - 1))[:n].contiguous()
        out = torch.empty((n, 22), dtype=torch.float64, device=dev)
        status = torch.empty((n,), dtype=torch.int32, device=dev)

        if args.path == "bates22":
            def step():
                eng.bates22(bt["prof"], bt["sub"], bt["dmcurve"], bt["scal"], out=out, status=status)
        else:
            # config 5: the profile of each candidate also feeds the Lyon features, with a
            # 128-bin DM array per candidate; one (n, 30) feature matrix per step
            _, dmrows = lyon_batch_torch(n, args.lp, args.ld, seed=20261020 + rank, device=dev)
            o8 = torch.empty((n, 8), dtype=torch.float64, device=dev)
            out = torch.empty((n, 30), dtype=torch.float64, device=dev)

            def step():
                eng.lyon8(bt["prof"], dmrows, out=o8)
                eng.bates22(bt["prof"], bt["sub"], bt["dmcurve"], bt["scal"], out=out22,
                            status=status)
                out[:, :8].copy_(o8)
                out[:, 8:].copy_(out22)

            out22 = torch.empty((n, 22), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # step-duration events on the kernels' own stream
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        step()
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps

    if dist_on:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        if backend == "nccl":
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        else:
            tc = t.cpu()
            dist.all_reduce(tc, op=dist.ReduceOp.MAX)
            t = tc
        elapsed, kern_ms_max = float(t[0]), float(t[1])
    else:
        kern_ms_max = kern_ms

    total_rows = n * world * args.steps
    value = total_rows / elapsed
    common = {
        "value": value,
        "unit": "candidates/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "data": "synthetic (SURVEY.md §8(d) recipe, generated on device)",
    }
    if args.path == "lyon8":
        bytes_per_launch = n * (args.lp + args.ld + 8 * 8)
        achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
        traffic = load_traffic(f"lyon8_u8_{args.lp}x{args.ld}_n{n}_pmc.json")
        result = {
            "metric": "candidates/sec (8-feature path, 128-bin)",
            **common,
            "dtype": "u8->int64/f64",
            "config": {
                "workload": f"config 2: {n} synthetic candidates per GPU, {args.lp}-bin profile + "
                            f"{args.ld}-bin DM, 8 Lyon moment features (pfe_lyon8_u8)",
                "candidates_per_gpu": n,
                "profile_bins": args.lp,
                "dm_bins": args.ld,
                "parallelism": f"candidate shards x{world}, no collective",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "pfe::lyon8_u8_fast3<128, 2>",
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "avg_kernel_ms": kern_ms,
                "avg_kernel_ms_max_over_ranks": kern_ms_max,
            },
        }
    elif args.path == "pfd":
        npart, nsub, L = pfd_shape
        bytes_per_launch = n * (npart * nsub * L * 8 + nsub * 8 + 8 * 8 + 8 * 8 + 4)
        achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
        result = {
            "metric": "candidates/sec (PFD dmprof path)",
            **common,
            "dtype": "f64 (DM-curve statistics f32, as numpy)",
            "config": {
                "workload": f"{n} synthetic PRESTO folds per GPU ({npart} parts x {nsub} "
                            f"sub-bands x {L} bins): dedispersion, 0..255 profile, 100-DM "
                            f"chi^2 curve, 8 Lyon features (pfe_pfd_dmprof)",
                "candidates_per_gpu": n,
                "fold_shape": list(pfd_shape),
                "parallelism": f"candidate shards x{world}, no collective",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": None,
                "kernel": "pfe::k_pfd_dmprof",
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "avg_kernel_ms": kern_ms,
                "avg_kernel_ms_max_over_ranks": kern_ms_max,
            },
        }
    elif args.path == "pfd22":
        npart, nsub, L = pfd_shape
        result = {
            "metric": "candidates/sec (PFD 22-score path)",
            **common,
            "dtype": "f64",
            "config": {
                "workload": f"{n} synthetic PRESTO folds per GPU ({npart} parts x {nsub} "
                            f"sub-bands x {L} bins): PFDFile.compute, 22 scores "
                            f"(pfe_pfd_bates22)",
                "candidates_per_gpu": n,
                "fold_shape": list(pfd_shape),
                "parallelism": f"candidate shards x{world}, no collective",
            },
            "roofline": {
                "bound": "fp64-valu",
                "achieved": None,
                "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": None,
                "traffic": None,
                "note": "operation count of the PFD 22-score path not frozen yet; the "
                        "fits are the 22-score path's (see --path bates22)",
                "kernel": "pfe_pfd_bates22 (9 kernels, one step)",
                "avg_step_ms": kern_ms,
                "avg_step_ms_max_over_ranks": kern_ms_max,
            },
        }
    else:
        ops = load_ops_per_candidate()
        achieved = (ops * n / (kern_ms * 1e-3) / 1e12) if ops else None
        all30 = args.path == "all30"
        result = {
            "metric": ("candidates/sec (8+22-feature path, 128-bin)" if all30
                       else "candidates/sec (22-score path, 128-bin)"),
            **common,
            "dtype": "f64",
            "config": {
                "workload": (f"config 5 shard: {n} synthetic candidates per GPU, {args.lp}-bin "
                             f"profile + {args.ld}-bin DM array, 16x{args.lp} sub-bands, 128-point "
                             f"DM curve, 8 Lyon + 22 Bates features into one (n, 30) matrix "
                             f"(pfe_lyon8_u8 + pfe_bates22)") if all30 else
                            (f"config 3 shape: {n} synthetic candidates per GPU, {args.lp}-bin "
                             f"profile, 16x{args.lp} sub-bands, 128-point DM curve, 22 Bates "
                             f"scores (pfe_bates22)"),
                "candidates_per_gpu": n,
                "profile_bins": args.lp,
                "parallelism": f"candidate shards x{world}, no collective",
            },
            "roofline": {
                "bound": "fp64-valu",
                "achieved": achieved,
                "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": (achieved / FP64_PEAK_TFLOPS) if achieved else None,
                "traffic": None,
                "kernel": ("pfe_lyon8_u8 + pfe_bates22, one step" if all30
                           else "pfe_bates22 (8 kernels, one step)"),
                "algorithmic_ops_per_candidate": ops,
                "avg_step_ms": kern_ms,
                "avg_step_ms_max_over_ranks": kern_ms_max,
            },
        }
    if args.gather and dist_on:
        # the optional reassembly step (RCCL all-gather of the n*world x 8 fp64 matrix over
        # xGMI), timed on its own, outside the headline step
        from pulsarfeatureextractor_amd.distributed import gather_rows

        gather_rows(out, n * world)
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        full = gather_rows(out, n * world)
        torch.cuda.synchronize()
        dist.barrier()
        gms = (time.perf_counter() - g0) * 1e3
        result["gather"] = {"ms": gms, "bytes_received_per_rank": int(full.numel() * 8 * (world - 1) / world),
                            "collective": "all_gather_into_tensor (RCCL)"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_sample > 0:
        if args.path == "lyon8":
            result["cpu_baseline"] = cpu_baseline_lyon8(args.lp, args.ld, args.cpu_sample)
            omp = cpu_baseline_lyon8_omp(args.lp, args.ld)
            if omp is not None:
                result["cpu_baseline_multicore"] = omp
        elif args.path == "pfd":
            result["cpu_baseline"] = cpu_baseline_pfd(pfd_shape, args.cpu_sample)
        elif args.path == "pfd22":
            result["cpu_baseline"] = cpu_baseline_pfd22(pfd_shape, args.cpu_sample)
        elif args.path == "all30":
            b = cpu_baseline_bates22(args.lp, args.cpu_sample)
            l8 = cpu_baseline_lyon8(args.lp, args.ld, 8000)
            v = 1.0 / (1.0 / b["value"] + 1.0 / l8["value"])
            result["cpu_baseline"] = {"value": v, "unit": "candidates/sec", "cores": 1,
                                      "kind": "port",
                                      "sample": f"{b['sample']}; plus {l8['sample']}; "
                                                f"combined per-candidate time"}
        else:
            result["cpu_baseline"] = cpu_baseline_bates22(args.lp, args.cpu_sample)
        if args.path in ("bates22", "all30") and not args.no_cpu_multicore:
            result["cpu_baseline_multicore"] = cpu_baseline_bates22_mp(args.lp)
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
