#!/bin/bash
# the GPU test files after test_bates22_gpu.py, the default bench line, the PFD / 22-score
# solve statistics (instrumented build) and the 2-rank gloo rehearsal of the N>1 bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_candidate_api_gpu.py tests/test_capi_gpu.py tests/test_cli_gpu.py tests/test_label_gpu.py tests/test_lyon8_gpu.py tests/test_pfd22_gpu.py tests/test_pfd_gpu.py tests/test_subband_gpu.py > gpurun_out/r03_gpu_suite_b.txt 2>&1 || { tail -60 gpurun_out/r03_gpu_suite_b.txt; exit 1; }
tail -3 gpurun_out/r03_gpu_suite_b.txt
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_default.json 2> gpurun_out/r03_bench_default.err || { tail -30 gpurun_out/r03_bench_default.err; exit 1; }
cat gpurun_out/r03_bench_default.json
timeout -k 10 300 python -u tools/lm_profile.py --path pfd22 --solver batched --n 4096 > gpurun_out/r03_lmprof_pfd22.json 2> gpurun_out/r03_lmprof_pfd22.err || { tail -20 gpurun_out/r03_lmprof_pfd22.err; exit 1; }
PFE_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 5 --warmup 1 --config5-n 1000000 > gpurun_out/r03_rehearse_2rank_gloo.json 2> gpurun_out/r03_rehearse_2rank_gloo.err || { tail -30 gpurun_out/r03_rehearse_2rank_gloo.err; exit 1; }
tail -1 gpurun_out/r03_rehearse_2rank_gloo.json
