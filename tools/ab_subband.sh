#!/bin/bash
# Sub-band kernel A/B: bit-identity of every output against the previous build, then the
# config-4 bench alternating three builds (GPU box, repo root).
set -o pipefail
mkdir -p gpurun_out
L=$PWD/pulsarfeatureextractor_amd/lib
export PYTHONUNBUFFERED=1
PFE_LIBRARY=$L/libpfe_pre.so timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_a.npz > gpurun_out/ab_dump.log 2>&1 &&
timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_b.npz >> gpurun_out/ab_dump.log 2>&1 &&
python tools/lib_outputs.py compare gpurun_out/out_a.npz gpurun_out/out_b.npz > gpurun_out/ab_compare.txt 2>&1; grep sub gpurun_out/ab_compare.txt; tail -1 gpurun_out/ab_compare.txt
for r in 1 2; do
  for lib in libpfe_pre.so libpfe.so libpfe_sub2.so; do
    PFE_LIBRARY=$L/$lib timeout -k 10 120 python bench.py --path subband --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_sub.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab_sub.json').readlines()[-1]);print('$lib',round(d['value']/1e6,1),'M/s kernel',round(d['roofline']['avg_kernel_ms'],3),'ms')"
  done
done
