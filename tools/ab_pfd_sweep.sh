#!/bin/bash
# PFD DM-sweep A/B (GPU box, repo root): bit-identity of every output of the previous build
# (libpfe_pre.so) and this one, then bench --path pfd alternating the two builds.
set -o pipefail
mkdir -p gpurun_out
L=$PWD/pulsarfeatureextractor_amd/lib
export PYTHONUNBUFFERED=1
PFE_LIBRARY=$L/libpfe_pre.so timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_a.npz > gpurun_out/ab_dump.log 2>&1 &&
timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_b.npz >> gpurun_out/ab_dump.log 2>&1 || exit 1
python tools/lib_outputs.py compare gpurun_out/out_a.npz gpurun_out/out_b.npz > gpurun_out/ab_compare.txt 2>&1; grep pfd gpurun_out/ab_compare.txt; tail -1 gpurun_out/ab_compare.txt
for r in 1 2; do
  for lib in libpfe_pre.so libpfe.so; do
    PFE_LIBRARY=$L/$lib timeout -k 10 180 python bench.py --path pfd --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_pfd.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab_pfd.json').readlines()[-1]);print('$lib',round(d['value']/1e6,3),'M folds/s kernel',round(d['roofline']['avg_kernel_ms'],3),'ms frac',round(d['roofline']['frac'],3))"
  done
done
