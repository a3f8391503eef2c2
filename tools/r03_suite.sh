#!/bin/bash
# the whole GPU suite on the product build (parity log of any stable-row allowance used)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PFE_PARITY_LOG=gpurun_out/r03_parity_slack.jsonl timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03_gpu_suite.txt 2>&1 || { tail -60 gpurun_out/r03_gpu_suite.txt; exit 1; }
tail -3 gpurun_out/r03_gpu_suite.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.txt 2>&1 || { cat gpurun_out/r03_smoke.txt; exit 1; }
cat gpurun_out/r03_smoke.txt
