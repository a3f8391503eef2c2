#!/bin/bash
# One-chunk DataBlock rows (nDM 30 / 33 / 60 / 8): next-row prefetch A/B (GPU box, repo root)
#   tools/r05_ab_l8pref.sh <lib> [<lib> ...]      (1M rows each, alternating twice)
set -o pipefail
L=$PWD/pulsarfeatureextractor_amd/lib
for r in 1 2; do
  for lib in "$@"; do
    PFE_LIBRARY=$L/$lib timeout -k 10 300 python -u tools/lyon8_long_bench.py --n 1000000 --ld 3840,4224,7680,1024 \
      > gpurun_out/ab_l8p.jsonl 2>&1 || { tail -5 gpurun_out/ab_l8p.jsonl; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/ab_l8p.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$lib', d['ld'], round(d['avg_kernel_ms'],4), 'ms', round(d['frac_of_8TBps'],4))"
  done
done
