#!/bin/bash
# A/B: enorm fast path, contracted gtol test, squared norm-loss test (libpfe.so) vs the
# previous build (libpfe_rcp2.so); golden dump; the whole GPU suite
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/ab_lib_bates.sh pulsarfeatureextractor_amd/lib/libpfe_rcp2.so pulsarfeatureextractor_amd/lib/libpfe.so > gpurun_out/r03_ab_rcp3.txt 2>&1 || { cat gpurun_out/r03_ab_rcp3.txt; tail gpurun_out/ab_lib.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_ab_rcp3.txt
timeout -k 10 200 python -u tools/golden_dump.py gpurun_out/r03_golden_rcp3.npz > gpurun_out/r03_dump_rcp3.log 2>&1 || { tail -20 gpurun_out/r03_dump_rcp3.log; exit 1; }
PFE_PARITY_LOG=gpurun_out/r03_parity_slack.jsonl timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03_gpu_suite.txt 2>&1 || { tail -60 gpurun_out/r03_gpu_suite.txt; exit 1; }
tail -3 gpurun_out/r03_gpu_suite.txt
