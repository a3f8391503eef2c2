#!/bin/bash
# Lyon-8 headline kernel: grid cap A/B (handle option lyon8_blocks), alternating on one box
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for B in 8192 16384 4096; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --option lyon8_blocks=$B > gpurun_out/ab_l8.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab_l8.json').readlines()[-1]);print('blocks $B', round(d['roofline']['avg_kernel_ms'],4), 'ms', round(d['roofline']['frac'],4))"
  done
done
