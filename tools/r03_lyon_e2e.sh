#!/bin/bash
# Lyon-8 long-row kernels (tests + timing at the PHCX DataBlock shape), then the streamed
# files-to-scores product path on 50k synthetic PHCX files.
set -e
set -o pipefail
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lyon8_gpu.py > gpurun_out/r03_lyon8_tests.txt 2>&1 || { tail -40 gpurun_out/r03_lyon8_tests.txt; exit 1; }
tail -2 gpurun_out/r03_lyon8_tests.txt
timeout -k 10 200 python -u tools/lyon8_long_bench.py > gpurun_out/r03_lyon8_long.jsonl 2> gpurun_out/r03_lyon8_long.err || { tail -20 gpurun_out/r03_lyon8_long.err; exit 1; }
cat gpurun_out/r03_lyon8_long.jsonl
timeout -k 10 600 python -u tools/e2e_bench.py --n 50000 --mode stream --workers 16 --batch 8192 > gpurun_out/r03_e2e_stream.json 2> gpurun_out/r03_e2e_stream.err || { tail -30 gpurun_out/r03_e2e_stream.err; exit 1; }
cat gpurun_out/r03_e2e_stream.json
