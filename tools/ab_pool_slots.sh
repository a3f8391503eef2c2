#!/bin/bash
# Slot pools sized by the batch (GPU box, repo root): bit-identity of libpfe_pre.so and this
# build, then the PFD 22-score bench (32k folds: a batch that does not fill the waves) and the
# 22-score bench (1M: one that does), alternating the two builds.
set -o pipefail
mkdir -p gpurun_out
L=$PWD/pulsarfeatureextractor_amd/lib
export PYTHONUNBUFFERED=1
PFE_LIBRARY=$L/libpfe_pre.so timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_a.npz > gpurun_out/ab_dump.log 2>&1 &&
timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_b.npz >> gpurun_out/ab_dump.log 2>&1 || exit 1
python tools/lib_outputs.py compare gpurun_out/out_a.npz gpurun_out/out_b.npz > gpurun_out/ab_compare.txt 2>&1; tail -1 gpurun_out/ab_compare.txt
for r in 1 2; do
  for lib in libpfe_pre.so libpfe.so; do
    for p in pfd22 bates22; do
      PFE_LIBRARY=$L/$lib timeout -k 10 200 python bench.py --path $p --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ab_ps.json 2>gpurun_out/ab_ps.err || exit 1
      python -c "import json;d=json.loads(open('gpurun_out/ab_ps.json').readlines()[-1]);print('$lib $p',round(d['value']),round(d['ms_per_step'],1))"
    done
  done
done
