#!/bin/bash
# the whole GPU suite + smoke on the final tree
set -e
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03z_gpu_suite.txt 2>&1 || { tail -60 gpurun_out/r03z_gpu_suite.txt; exit 1; }
tail -1 gpurun_out/r03z_gpu_suite.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
