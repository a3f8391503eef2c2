#!/usr/bin/env python3
"""End-to-end throughput of the batched ScoreGenerator path: directory of PHCX files ->
native parse -> pfe_bates22 / pfe_lyon8 on the GPU -> score text, phase by phase.

  python tools/e2e_bench.py --n 4000 [--dir /tmp/pfe_e2e] [--workers 16] [--mode phases|stream]

The synthetic files follow SURVEY.md §8(d) (128-bin profile, 16x128 sub-bands, a
128 x 128 DataBlock per section, i.e. 128 DM trials, so the DmIndex lists 128 DM values as a
real PHCX file lists one per DataBlock row).  Writing them is not timed.

--mode phases (default): parse everything, then score everything, phase by phase.
--mode stream: the product path, DataProcessor.processPHCXCollectively (22 scores) and
dmprofPHCX (8 Lyon features) -- batches of --batch files parsed by the native reader on a
helper thread one batch ahead of the GPU stage (pfe_phcx_pack into pinned slabs, libpfe on
them, pfe_format_rows), each batch's lines appended in discovery order; reports the wall
time, the native reader's own rate on the same files (parse only, and parse + pack) and the
process's peak RSS (run it in its own process so the peak is the streamed path's).
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _write(args):
    i, d = args
    from pulsarfeatureextractor_amd import phcx
    from pulsarfeatureextractor_amd.synth import bates_batch

    b = bates_batch(1, seed=7000 + i)
    rng = np.random.default_rng(i)
    curve = b["dmcurve"][0]
    blocks = (phcx.make_datablock(curve, rng), phcx.make_datablock(curve, rng))
    s = b["scal"][0]
    p = os.path.join(d, f"cand_{i:06d}.phcx.gz")
    phcx.write(p, profile=b["prof"][0], subbands=b["sub"][0], datablocks=blocks,
               dm_start=0.0, dm_end=200.0, n_dm_index=len(blocks[1]) // 128,
               period_s=float(s[0]) / 1000.0, snr=float(s[1]), dm=float(s[2]), width=float(s[3]))
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4000)
    ap.add_argument("--dir", default="/tmp/pfe_e2e_r3")
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--mode", choices=["phases", "stream"], default="phases")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--ramp", type=int, default=1, help="ramped batch sizes at both ends (1, default) or not (0)")
    ap.add_argument("--unique", type=int, default=0,
                    help="write this many distinct files and hard-link them up to --n paths "
                         "(500k-file runs without 15 GB of distinct data; every path is still "
                         "opened, inflated and parsed)")
    ap.add_argument("--depth", default="2",
                    help="GPU pipeline depths to time, comma-separated (DataProcessor gpu_depth)")
    ap.add_argument("--gpus", default="1",
                    help="stream mode: shard counts to time, comma-separated (DataProcessor "
                         "gpus=N: N spawned workers, each on GPU r %% visible GPUs, the host "
                         "threads split between them)")
    args = ap.parse_args()
    os.makedirs(args.dir, exist_ok=True)
    have = sorted(f for f in os.listdir(args.dir) if f.endswith(".phcx.gz"))
    if len(have) < args.n:
        u = args.unique if 0 < args.unique < args.n else args.n
        with ProcessPoolExecutor(args.workers) as ex:
            list(ex.map(_write, [(i, args.dir) for i in range(u)], chunksize=64))
        for i in range(u, args.n):
            dst = os.path.join(args.dir, f"cand_{i:06d}.phcx.gz")
            if not os.path.exists(dst):
                os.link(os.path.join(args.dir, f"cand_{i % u:06d}.phcx.gz"), dst)
    from pulsarfeatureextractor_amd import processor, writers
    from pulsarfeatureextractor_amd.candidate import get_engine

    if args.mode == "stream":
        import resource
        import tempfile

        from pulsarfeatureextractor_amd._native import PhcxBatch

        paths = processor.discover(args.dir, [processor.PHCX_RE])
        nfiles = len(paths)
        res = {"mode": "stream", "files": nfiles, "batch": args.batch, "workers": args.workers}
        # the native reader alone on the same files (page cache warm after the first pass)
        for rep in range(2):
            t0 = time.perf_counter()
            for s0 in range(0, nfiles, args.batch):
                b = PhcxBatch(paths[s0:s0 + args.batch], threads=args.workers)
                b.close()
            res["reader_parse_files_per_s"] = nfiles / (time.perf_counter() - t0)
        t0 = time.perf_counter()
        for s0 in range(0, nfiles, args.batch):
            b = PhcxBatch(paths[s0:s0 + args.batch], threads=args.workers)
            inf = b.infos()
            b.pack(np.arange(len(inf)), lp=128, nsub_lsb=(16, 128), ndm=128,
                   threads=args.workers)
            b.close()
        res["reader_parse_pack_files_per_s"] = nfiles / (time.perf_counter() - t0)
        eng = get_engine(0)
        texts = {}
        runs = [(int(d), 1) for d in args.depth.split(",")]
        runs += [(int(args.depth.split(",")[-1]), int(g)) for g in args.gpus.split(",") if int(g) > 1]
        for depth, g in runs:
            for kind in ("scores", "dmprof"):
                out = os.path.join(tempfile.mkdtemp(), "scores.csv")
                dp = processor.DataProcessor(engine=eng, workers=args.workers,
                                             log=lambda *a: None, batch=args.batch,
                                             gpu_depth=depth, ramp=bool(args.ramp), gpus=g)
                t0 = time.perf_counter()
                if kind == "scores":
                    dp.processPHCXCollectively(args.dir, False, out, False, False, False)
                else:
                    dp.dmprofPHCX(args.dir, False, out, False, False)
                wall = time.perf_counter() - t0
                with open(out) as f:
                    text = f.read()
                same = texts.setdefault(kind, text) == text
                res[f"{kind}_depth{depth}" + (f"_gpus{g}" if g > 1 else "")] = {
                                               "wall_s": wall, "files_per_s": nfiles / wall,
                                               "lines": text.count("\n"),
                                               "text_identical_to_first_depth": same,
                                               "metrics": dp.metrics}
        res["peak_rss_MB"] = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024
        d0 = args.depth.split(",")[-1]
        res["frac_of_reader"] = (res[f"scores_depth{d0}"]["files_per_s"] /
                                 res["reader_parse_pack_files_per_s"])
        print(json.dumps(res))
        return
    eng = get_engine(0)
    paths = processor.discover(args.dir, [processor.PHCX_RE])[: args.n]
    res = {"files": len(paths)}
    t0 = time.perf_counter()
    parsed = processor.parse_all(paths, args.workers, native=True)
    t1 = time.perf_counter()
    cands = [c for c, e in parsed if c is not None]
    sc, errs = processor.score_bates(cands, eng)
    t2 = time.perf_counter()
    lines = [writers.score_line(c.path, sc[j]) for j, c in enumerate(cands) if errs[j] is None]
    t3 = time.perf_counter()
    ly = processor.score_lyon8(cands, eng)
    t4 = time.perf_counter()
    res.update({
        "parse_native_s": t1 - t0, "parse_files_per_s": len(paths) / (t1 - t0),
        "bates22_s": t2 - t1, "bates22_cand_per_s": len(cands) / (t2 - t1),
        "write_lines_s": t3 - t2, "lyon8_s": t4 - t3,
        "e2e_22score_files_per_s": len(paths) / (t3 - t0),
        "scored": len(lines), "lyon_rows": int(np.isfinite(ly[:, 0]).sum()),
        "workers": args.workers,
    })
    n_py = min(200, len(paths))
    t5 = time.perf_counter()
    processor.parse_all(paths[:n_py], 1, native=False)
    res["parse_python_1core_files_per_s"] = n_py / (time.perf_counter() - t5)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
