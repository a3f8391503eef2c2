#!/bin/bash
# A/B of the Lyon-8 stream kernel's burst (candidate groups per wave step, handle option
# lyon8_burst), alternating runs on one GPU.
for r in 1 2; do
  for v in ${BURSTS:-1 2 4}; do
    timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-extra --option lyon8_burst=$v \
      | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('burst $v', round(d['roofline']['avg_kernel_ms'],4), 'ms', round(d['roofline']['achieved']), 'GB/s', round(d['value']/1e9,2), 'Gcand/s')"
  done
done
