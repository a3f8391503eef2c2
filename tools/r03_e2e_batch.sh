#!/bin/bash
# streamed files-to-scores at three batch sizes (50k synthetic PHCX files)
set -e
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for B in 8192 16384 32768; do
  timeout -k 10 400 python -u tools/e2e_bench.py --n 50000 --mode stream --workers 16 --batch $B > gpurun_out/r03_e2e_b$B.json 2> gpurun_out/r03_e2e_b$B.err || { tail -20 gpurun_out/r03_e2e_b$B.err; exit 1; }
  cat gpurun_out/r03_e2e_b$B.json
done
