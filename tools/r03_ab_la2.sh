#!/bin/bash
# LA quotient removal in the pooled qrfac / Q^T f (libpfe.so) vs the previous build
# (libpfe_base.so): 22-score parity tests on the new build, then the alternating A/B.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bates22_gpu.py tests/test_pfd22_gpu.py tests/test_all30_gpu.py > gpurun_out/r03_la6_tests.txt 2>&1 || { tail -40 gpurun_out/r03_la6_tests.txt; exit 1; }
tail -2 gpurun_out/r03_la6_tests.txt
bash tools/ab_lib_bates.sh pulsarfeatureextractor_amd/lib/libpfe_base.so pulsarfeatureextractor_amd/lib/libpfe.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_ab_la6.txt
