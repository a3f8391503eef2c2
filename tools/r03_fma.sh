#!/bin/bash
# FMA-contracted solver linear algebra (libpfe.so) vs the uncontracted build (libpfe_nofma.so):
# parity tests on the FMA build, golden dump for the envelope report, then the alternating
# 22-score bench; plus the Lyon / sub-band / CLI / plug-in API tests and the e2e stream.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lyon8_gpu.py tests/test_subband_gpu.py tests/test_cli_gpu.py tests/test_label_gpu.py tests/test_candidate_api_gpu.py > gpurun_out/r03_t1.txt 2>&1 || { tail -40 gpurun_out/r03_t1.txt; exit 1; }
tail -2 gpurun_out/r03_t1.txt
timeout -k 10 180 python -u tools/golden_dump.py gpurun_out/r03_golden_gpu_fma.npz > gpurun_out/r03_dumps.log 2>&1 || { tail -20 gpurun_out/r03_dumps.log; exit 1; }
timeout -k 10 180 python -u tools/fresh_dump.py gpurun_out/r03_fresh_gpu_fma.npz >> gpurun_out/r03_dumps.log 2>&1 || { tail -20 gpurun_out/r03_dumps.log; exit 1; }
bash tools/ab_lib_bates.sh pulsarfeatureextractor_amd/lib/libpfe_nofma.so pulsarfeatureextractor_amd/lib/libpfe.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_ab_fma.txt
timeout -k 10 300 python -u tools/lm_profile.py --path pfd22 --solver batched --n 1024 > gpurun_out/r03_lmprof_pfd22.json 2> gpurun_out/r03_lmprof_pfd22.err || { tail -20 gpurun_out/r03_lmprof_pfd22.err; exit 1; }
timeout -k 10 600 python -u tools/e2e_bench.py --n 32768 --mode stream --workers 16 --batch 8192 > gpurun_out/r03_e2e_stream.json 2> gpurun_out/r03_e2e_stream.err || { tail -30 gpurun_out/r03_e2e_stream.err; exit 1; }
cat gpurun_out/r03_e2e_stream.json
