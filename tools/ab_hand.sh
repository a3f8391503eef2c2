#!/bin/bash
# A/B of the LM hand-over scratch (handle option handover=0 re-evaluates): parity tests, then bates22/pfd22
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bates22_gpu.py tests/test_pfd22_gpu.py > gpurun_out/t_hand.log 2>&1 || { tail -30 gpurun_out/t_hand.log; exit 1; }
tail -2 gpurun_out/t_hand.log
for v in 1 0; do
  timeout -k 10 200 python bench.py --path bates22 --option handover=$v > gpurun_out/b_hand$v.json 2>gpurun_out/b_hand.err || exit 1
  timeout -k 10 200 python bench.py --path pfd22 --option handover=$v > gpurun_out/b_hand${v}_pfd22.json 2>>gpurun_out/b_hand.err || exit 1
done
for f in gpurun_out/b_hand*.json; do python -c "import json,sys;d=json.load(open('$f'));print('$f',round(d['value']),round(d['ms_per_step'],1))"; done
