#!/bin/bash
# One-chunk 32-leaf DataBlock rows (nDM 30, two rows per wave): A/B of two libraries, 1M rows,
# alternating three times:  tools/r05_ab_l8pair.sh <libA> <libB>
set -o pipefail
L=$PWD/pulsarfeatureextractor_amd/lib
for r in 1 2 3; do
  for lib in "$@"; do
    PFE_LIBRARY=$L/$lib timeout -k 10 200 python -u tools/lyon8_long_bench.py --n 1000000 --ld 3840 \
      > gpurun_out/ab_l8pr.jsonl 2>&1 || { tail -5 gpurun_out/ab_l8pr.jsonl; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/ab_l8pr.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$lib', d['ld'], round(d['avg_kernel_ms'],4), 'ms', round(d['frac_of_8TBps'],4))"
  done
done
