#!/bin/bash
# Phase split of k_pfd_dmprof4 (GPU box, repo root): the product build against instrumented
# builds without the DM sweep (libpfe_probe1.so) and without the wave-0 tail (probe2).
set -o pipefail
mkdir -p gpurun_out
L=$PWD/pulsarfeatureextractor_amd/lib
export PYTHONUNBUFFERED=1
for lib in libpfe.so libpfe_probe1.so libpfe_probe2.so; do
  PFE_LIBRARY=$L/$lib timeout -k 10 180 python bench.py --path pfd --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/probe_pfd.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/probe_pfd.json').readlines()[-1]);print('$lib',round(d['value']/1e6,3),'M folds/s kernel',round(d['roofline']['avg_kernel_ms'],3),'ms')"
done
