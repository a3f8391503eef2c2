#!/bin/bash
# Full GPU test suite + smoke (run on the GPU box from the repo root).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r02_gpu_suite.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/r02_gpu_suite.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids
