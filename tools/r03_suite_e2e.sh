#!/bin/bash
# GPU suite, then the streamed files-to-scores path on 32k synthetic PHCX files
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03_gpu_suite.txt 2>&1 || { tail -60 gpurun_out/r03_gpu_suite.txt; exit 1; }
tail -3 gpurun_out/r03_gpu_suite.txt
timeout -k 10 600 python -u tools/e2e_bench.py --n 32768 --mode stream --workers 16 --batch 8192 > gpurun_out/r03_e2e_stream.json 2> gpurun_out/r03_e2e_stream.err || { tail -30 gpurun_out/r03_e2e_stream.err; exit 1; }
cat gpurun_out/r03_e2e_stream.json
