#!/bin/bash
# GPU-box profiling recipe (run from the repo root on the MI355X box):
#   1. kernel trace + stats of the headline bench       -> gpurun_out/prof_trace
#   2. PMC pass FETCH_SIZE (own pass)                    -> gpurun_out/prof_fetch
#   3. PMC pass WRITE_SIZE (own pass)                    -> gpurun_out/prof_write
#   4. kernel trace + stats of the 22-score path         -> gpurun_out/prof_bates
# Every step has its own time limit; the script stops at the first failure.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${N:-10000000}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o trace -- \
  python3 bench.py --steps 20 --warmup 3 --n $N --no-cpu-baseline > gpurun_out/prof_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o pmc -- \
  python3 bench.py --steps 5 --warmup 1 --n $N --no-cpu-baseline > gpurun_out/prof_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o pmc -- \
  python3 bench.py --steps 5 --warmup 1 --n $N --no-cpu-baseline > gpurun_out/prof_write.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bates -o trace -- \
  python3 tools/bates_throughput.py --n 100000 --reps 2 > gpurun_out/prof_bates.log 2>&1
echo profile-done
