#!/bin/bash
# k_gdg8g with 48 vs 32 fit slots per wave (GPU box, repo root): bit-identity of every
# output of libpfe_pre.so and this build, then the 22-score bench alternating the two,
# concurrent score groups and serialised.
set -o pipefail
mkdir -p gpurun_out
L=$PWD/pulsarfeatureextractor_amd/lib
export PYTHONUNBUFFERED=1
PFE_LIBRARY=$L/libpfe_pre.so timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_a.npz > gpurun_out/ab_dump.log 2>&1 &&
timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_b.npz >> gpurun_out/ab_dump.log 2>&1 || exit 1
python tools/lib_outputs.py compare gpurun_out/out_a.npz gpurun_out/out_b.npz > gpurun_out/ab_compare.txt 2>&1; tail -1 gpurun_out/ab_compare.txt
for r in 1 2; do
  for lib in libpfe_pre.so libpfe.so; do
    for opt in serial=0 serial=1; do
      PFE_LIBRARY=$L/$lib timeout -k 10 200 python bench.py --path bates22 --steps 4 --warmup 1 --no-cpu-baseline --option $opt > gpurun_out/ab_wpe.json 2>gpurun_out/ab_wpe.err || exit 1
      python -c "import json;d=json.loads(open('gpurun_out/ab_wpe.json').readlines()[-1]);print('$lib $opt',round(d['value']),round(d['ms_per_step'],1))"
    done
  done
done
