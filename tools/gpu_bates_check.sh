#!/bin/bash
# Bates/PFD 22-score parity tests, then one bench line each (bates22, pfd22)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bates22_gpu.py tests/test_pfd22_gpu.py tests/test_cli_gpu.py > gpurun_out/t_bates.log 2>&1 || { tail -40 gpurun_out/t_bates.log; exit 1; }
tail -2 gpurun_out/t_bates.log
timeout -k 10 200 python bench.py --path bates22 > gpurun_out/b_bates22.json 2>gpurun_out/b_bates.err || exit 1
timeout -k 10 200 python bench.py --path pfd22 > gpurun_out/b_pfd22.json 2>>gpurun_out/b_bates.err || exit 1
for f in gpurun_out/b_bates22.json gpurun_out/b_pfd22.json; do python -c "import json;d=json.load(open('$f'));print('$f',round(d['value']),round(d['ms_per_step'],1))"; done
