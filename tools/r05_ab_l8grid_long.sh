#!/bin/bash
# Grid cap A/B for the DataBlock-length Lyon-8 kernels (GPU box, repo root): 1M rows at
# ld = 16384 / 15360 / 12800 / 9216, PFE_OPT_LYON8_BLOCKS 16384 vs the default, twice.
set -o pipefail
for r in 1 2; do
  for b in 16384 131072; do
    timeout -k 10 300 python -u tools/lyon8_long_bench.py --n 1000000 --ld 16384,15360,12800,9216 \
      --opt lyon8_blocks=$b > gpurun_out/ab_l8gl.jsonl 2>&1 || { tail -5 gpurun_out/ab_l8gl.jsonl; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/ab_l8gl.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('blocks $b', d['ld'], round(d['avg_kernel_ms'],4), 'ms', round(d['frac_of_8TBps'],4))"
  done
done
