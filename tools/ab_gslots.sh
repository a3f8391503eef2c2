#!/bin/bash
# A/B of the pooled kernels' slots per wave (handle option gslots) on the 22-score bench
set -o pipefail
mkdir -p gpurun_out
for g in 16 24 32; do
  timeout -k 10 200 python bench.py --path bates22 --steps 10 --warmup 2 --no-cpu-baseline --option gslots=$g > gpurun_out/b_gs$g.json 2>gpurun_out/b_gs.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b_gs$g.json'));print('gslots $g',round(d['value']),round(d['ms_per_step'],1))"
done
