#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/diag_unsupported.py > gpurun_out/r03_diag.txt 2>&1 || { cat gpurun_out/r03_diag.txt; exit 1; }
cat gpurun_out/r03_diag.txt
timeout -k 10 180 python -u tools/golden_dump.py gpurun_out/r03_golden_gpu.npz > gpurun_out/r03_dumps.log 2>&1 || { tail -20 gpurun_out/r03_dumps.log; exit 1; }
timeout -k 10 180 python -u tools/fresh_dump.py gpurun_out/r03_fresh_gpu.npz >> gpurun_out/r03_dumps.log 2>&1 || { tail -20 gpurun_out/r03_dumps.log; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lyon8_gpu.py tests/test_cli_gpu.py tests/test_label_gpu.py tests/test_candidate_api_gpu.py > gpurun_out/r03_lyon_cli.txt 2>&1 || { tail -40 gpurun_out/r03_lyon_cli.txt; exit 1; }
tail -3 gpurun_out/r03_lyon_cli.txt
timeout -k 10 300 python -u tools/lm_profile.py --path pfd22 --solver batched --n 1024 > gpurun_out/r03_lmprof_pfd22.json 2> gpurun_out/r03_lmprof_pfd22.err || { tail -20 gpurun_out/r03_lmprof_pfd22.err; exit 1; }
timeout -k 10 600 python -u tools/e2e_bench.py --n 32768 --mode stream --workers 16 --batch 8192 > gpurun_out/r03_e2e_stream.json 2> gpurun_out/r03_e2e_stream.err || { tail -30 gpurun_out/r03_e2e_stream.err; exit 1; }
cat gpurun_out/r03_e2e_stream.json
