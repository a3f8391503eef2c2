#!/bin/bash
# Re-check of a restored tree (GPU box, repo root): the GPU suite + smoke, then the default
# bench line.  Each step has its own time limit; stop at the first failure.
set -e
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/r02_gpu_suite.sh
echo suite-done
timeout -k 10 400 python3 bench.py > gpurun_out/r02c_bench_default.json 2> gpurun_out/r02c_bench_default.err
echo bench-done
