#!/bin/bash
# Round 3, restored tree: full GPU suite, the default bench line, then the FMA A/B of the
# 22-score chain (libpfe.so = contracted solver linear algebra, libpfe_nofma.so = uncontracted)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PFE_PARITY_LOG=gpurun_out/r03_parity_slack.jsonl timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03_gpu_suite.txt 2>&1 || { tail -60 gpurun_out/r03_gpu_suite.txt; exit 1; }
tail -3 gpurun_out/r03_gpu_suite.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_default.json 2> gpurun_out/r03_bench_default.err || { tail -30 gpurun_out/r03_bench_default.err; exit 1; }
cat gpurun_out/r03_bench_default.json
bash tools/ab_lib_bates.sh pulsarfeatureextractor_amd/lib/libpfe_nofma.so pulsarfeatureextractor_amd/lib/libpfe.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_ab_fma.txt
timeout -k 10 300 python -u tools/lm_profile.py --path pfd22 --solver batched --n 4096 > gpurun_out/r03_lmprof_pfd22.json 2> gpurun_out/r03_lmprof_pfd22.err || { tail -20 gpurun_out/r03_lmprof_pfd22.err; exit 1; }
timeout -k 10 300 python -u tools/lm_profile.py --path bates22 --solver batched --n 20000 > gpurun_out/r03_lmprof_bates22.json 2> gpurun_out/r03_lmprof_bates22.err || { tail -20 gpurun_out/r03_lmprof_bates22.err; exit 1; }
