#!/bin/bash
# A/B of two libpfe builds on the 22-score bench (alternating, 1M resident candidates):
#   tools/ab_lib_bates.sh <libA.so> <libB.so> [path]
set -o pipefail
mkdir -p gpurun_out
P=${3:-bates22}
for r in 1 2; do
  for L in "$1" "$2"; do
    PFE_LIBRARY=$L timeout -k 10 200 python bench.py --path $P --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ab_lib.json 2>gpurun_out/ab_lib.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab_lib.json').readlines()[-1]);print('$(basename $L)',round(d['value']),round(d['ms_per_step'],1))"
  done
done
