#!/bin/bash
# reciprocal quotients in the solver's linear algebra (libpfe.so) vs the FMA-only build
# (libpfe_fma0.so), then the whole GPU suite on libpfe.so
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/ab_lib_bates.sh pulsarfeatureextractor_amd/lib/libpfe_fma0.so pulsarfeatureextractor_amd/lib/libpfe.so > gpurun_out/r03_ab_rcp.txt 2>&1 || { cat gpurun_out/r03_ab_rcp.txt; tail gpurun_out/ab_lib.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_ab_rcp.txt
PFE_PARITY_LOG=gpurun_out/r03_parity_slack.jsonl timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03_gpu_suite.txt 2>&1 || { tail -60 gpurun_out/r03_gpu_suite.txt; exit 1; }
tail -3 gpurun_out/r03_gpu_suite.txt
