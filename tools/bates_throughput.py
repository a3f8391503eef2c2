#!/usr/bin/env python3
"""Throughput of the 22-score path on device-resident synthetic batches (config 3 shape)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lp", type=int, default=128)
    ap.add_argument("--lib", default=None, help="alternative libpfe build (A/B runs)")
    ap.add_argument("--save", default=None, help="write scores/status to this .npz")
    args = ap.parse_args()
    import torch

    from pulsarfeatureextractor_amd import _native
    from pulsarfeatureextractor_amd._native import Engine
    from pulsarfeatureextractor_amd.synth import bates_batch

    base = bates_batch(4096, lp=args.lp, lsb=args.lp, seed=31)
    reps = (args.n + 4095) // 4096
    t = {k: torch.from_numpy(np.ascontiguousarray(np.concatenate([v] * reps)[: args.n])).cuda()
         for k, v in base.items()}
    if args.lib:
        _native._lib = _native.load_library(os.path.abspath(args.lib))
    eng = Engine(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    eng.set_stream(s.cuda_stream)
    out = torch.empty((args.n, 22), dtype=torch.float64, device="cuda")
    st = torch.empty((args.n,), dtype=torch.int32, device="cuda")
    eng.bates22(t["prof"][:4096], t["sub"][:4096], t["dmcurve"][:4096], t["scal"][:4096],
                out[:4096], st[:4096])
    torch.cuda.synchronize()
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        eng.bates22(t["prof"], t["sub"], t["dmcurve"], t["scal"], out, st)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    best = min(times)
    if args.save:
        np.savez_compressed(args.save, out=out.cpu().numpy(), status=st.cpu().numpy())
    print(json.dumps({"n": args.n, "lp": args.lp, "seconds": times,
                      "candidates_per_sec": args.n / best,
                      "failures": int(((st & 0xFF) != 0).sum().item())}))


if __name__ == "__main__":
    main()
