#!/bin/bash
# Headline kernel grid cap A/B (GPU box, repo root): config 2 at PFE_OPT_LYON8_BLOCKS =
# 16384 (default), 32768, 65536, alternating three times; one line per run.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for b in ${GRIDS:-16384 32768 65536}; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --option lyon8_blocks=$b \
      > gpurun_out/ab_l8grid.json 2> gpurun_out/ab_l8grid.err || { tail -5 gpurun_out/ab_l8grid.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_l8grid.json').readlines()[-1]);r=d['roofline'];print('blocks $b', round(d['value']/1e9,3),'G cand/s kernel',round(r['avg_kernel_ms'],4),'ms frac',round(r['frac'],4))"
  done
done
