#!/bin/bash
# Kernel trace of the 22-score path with the score groups serialised (option serial=1), so each
# kernel's duration is its own; then the all30 bench line.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b22 -o trace -- \
  python3 bench.py --path bates22 --steps 4 --warmup 1 --no-cpu-baseline --option serial=1 > gpurun_out/prof_b22.log 2>&1
timeout -k 10 300 python3 bench.py --path all30 > gpurun_out/b_all30.json 2>gpurun_out/b_all30.err
cat gpurun_out/b_all30.json
find gpurun_out/prof_b22 -name "*kernel_stats.csv"
