#!/bin/bash
# A/B of the Lyon-8 grid cap (handle option lyon8_blocks), alternating runs on one GPU.
for r in 1 2; do
  for b in ${BLOCKS:-2048 4096 8192}; do
    timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-extra --option lyon8_blocks=$b > /tmp/ab.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('/tmp/ab.json').readlines()[-1]); print('blocks $b', round(d['roofline']['avg_kernel_ms'],4), 'ms', round(d['roofline']['achieved']), 'GB/s')"
  done
done
