#!/bin/bash
# A/B of Lyon-8 kernel variants (PFE_LYON8_VARIANT), alternating runs on one GPU.
for r in 1 2; do
  for v in ${VARIANTS:-1 2}; do
    PFE_LYON8_VARIANT=$v timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline \
      | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('variant $v', round(d['roofline']['avg_kernel_ms'],4), 'ms', round(d['roofline']['achieved']), 'GB/s', round(d['value']/1e9,2), 'Gcand/s')"
  done
done
