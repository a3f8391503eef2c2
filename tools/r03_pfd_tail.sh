#!/bin/bash
# PFD tail rewrite: PFD parity tests, then the PFD 22-score bench line and its serialised trace
set -e
set -o pipefail
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pfd_gpu.py tests/test_pfd22_gpu.py tests/test_label_gpu.py > gpurun_out/r03_pfd_tests.txt 2>&1 || { tail -40 gpurun_out/r03_pfd_tests.txt; exit 1; }
tail -2 gpurun_out/r03_pfd_tests.txt
bash tools/r03_pfd22_trace.sh
