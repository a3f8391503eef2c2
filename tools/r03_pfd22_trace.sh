#!/bin/bash
# serialised kernel trace of the PFD 22-score path and its bench line (frozen op count)
set -e
set -o pipefail
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --path pfd22 --steps 3 --warmup 1 > gpurun_out/r03_bench_pfd22.json 2> gpurun_out/r03_bench_pfd22.err || { tail -20 gpurun_out/r03_bench_pfd22.err; exit 1; }
echo pfd22-bench-done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_prof_pfd22 -o trace -- \
  python3 bench.py --path pfd22 --steps 2 --warmup 1 --no-cpu-baseline --option serial=1 > gpurun_out/r03_prof_pfd22.log 2>&1
echo pfd22-trace-done
