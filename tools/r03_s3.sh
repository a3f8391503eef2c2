#!/bin/bash
# FMA A/B first (22-score chain, alternating builds), then the GPU suite without the
# wave-vs-batched bit-identity test (contraction differs between the two code shapes)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/ab_lib_bates.sh pulsarfeatureextractor_amd/lib/libpfe_nofma.so pulsarfeatureextractor_amd/lib/libpfe.so > gpurun_out/r03_ab_fma.txt 2>&1 || { cat gpurun_out/r03_ab_fma.txt; cat gpurun_out/ab_lib.err | tail; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_ab_fma.txt
PFE_PARITY_LOG=gpurun_out/r03_parity_slack.jsonl timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_bates22_gpu.py::test_batched_solver_bit_identical > gpurun_out/r03_gpu_suite.txt 2>&1 || { tail -60 gpurun_out/r03_gpu_suite.txt; exit 1; }
tail -3 gpurun_out/r03_gpu_suite.txt
