#!/usr/bin/env python3
"""Lyon-8 at the real PHCX shape: a 128-bin profile + the whole section-0 DataBlock
(nDM x 128 bytes) per candidate, 1M resident candidates per length, HIP-event timed on the
kernel's stream.  Prints one JSON object per DataBlock length.

  python tools/lyon8_long_bench.py [--n 1000000] [--ld 16384,15360] [--steps 10]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--lp", type=int, default=128)
    ap.add_argument("--ld", default="16384,15360")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--opt", action="append", default=[],
                    help="handle option name=value (e.g. lyon8_dm=1), repeatable")
    args = ap.parse_args()
    import torch

    from pulsarfeatureextractor_amd._native import Engine
    from pulsarfeatureextractor_amd.synth import lyon_batch_torch

    eng = Engine(0)
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    eng.set_stream(st.cuda_stream)
    opts = {k: int(v) for k, v in (o.split("=") for o in args.opt)}
    for k, v in opts.items():
        eng.set_option(k, v)
    for ld in (int(v) for v in args.ld.split(",")):
        prof, dm = lyon_batch_torch(args.n, args.lp, ld, seed=20261023, device="cuda")
        out = torch.empty((args.n, 8), dtype=torch.float64, device="cuda")
        for _ in range(2):
            eng.lyon8(prof, dm, out=out)
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        for a, b in evs:
            a.record(st)
            eng.lyon8(prof, dm, out=out)
            b.record(st)
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
        nb = (args.lp + ld + 64) * args.n
        print(json.dumps({"lp": args.lp, "ld": ld, "n": args.n, "opts": opts, "avg_kernel_ms": ms,
                          "candidates_per_s": args.n / ms * 1e3,
                          "algorithmic_GBps": nb / ms / 1e6, "frac_of_8TBps": nb / ms / 8e9}),
              flush=True)
        del prof, dm, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
