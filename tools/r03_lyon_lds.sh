#!/bin/bash
# Lyon-8 tests + long-row timing (pow2 and LDS-staged kernels)
set -e
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lyon8_gpu.py > gpurun_out/r03_lyon8_tests.txt 2>&1 || { tail -40 gpurun_out/r03_lyon8_tests.txt; exit 1; }
tail -2 gpurun_out/r03_lyon8_tests.txt
timeout -k 10 200 python -u tools/lyon8_long_bench.py --ld 16384,15360,14336,12288 > gpurun_out/r03_lyon8_long.jsonl 2> gpurun_out/r03_lyon8_long.err || { tail -20 gpurun_out/r03_lyon8_long.err; exit 1; }
cat gpurun_out/r03_lyon8_long.jsonl
