#!/bin/bash
# Instruction-cache counters of the 22-score kernels (one SQ pass; GPU box, repo root).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU SQ_WAIT_INST_ANY \
  --output-format csv -d gpurun_out/r02_icache -o pmc -- \
  python3 bench.py --path bates22 --n 262144 --steps 2 --warmup 1 --no-cpu-baseline --option serial=1 > gpurun_out/r02_icache.log 2>&1
echo icache-done
