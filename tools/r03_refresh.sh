#!/bin/bash
# refresh the secondary bench lines on the final round-3 build: 22 scores at 256 bins, PFD
# dmprof (8 features), 1M config-5 shard (all30)
set -e
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --path bates22 --lp 256 --steps 3 --warmup 1 --no-cpu-multicore > gpurun_out/r03_bench_b22_256.json 2> gpurun_out/r03_bench_b22_256.err || { tail -20 gpurun_out/r03_bench_b22_256.err; exit 1; }
tail -1 gpurun_out/r03_bench_b22_256.json | cut -c1-200
timeout -k 10 300 python3 bench.py --path pfd --steps 10 --warmup 2 > gpurun_out/r03_bench_pfd.json 2> gpurun_out/r03_bench_pfd.err || { tail -20 gpurun_out/r03_bench_pfd.err; exit 1; }
tail -1 gpurun_out/r03_bench_pfd.json | cut -c1-200
timeout -k 10 300 python3 bench.py --path all30 --steps 3 --warmup 1 > gpurun_out/r03_bench_all30.json 2> gpurun_out/r03_bench_all30.err || { tail -20 gpurun_out/r03_bench_all30.err; exit 1; }
tail -1 gpurun_out/r03_bench_all30.json | cut -c1-200
