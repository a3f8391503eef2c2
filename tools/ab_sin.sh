#!/bin/bash
# Restated small-argument sin: bit-identity against the previous build, then the 22-score
# bench alternating (previous, this build, this build at 2 waves per SIMD for k_sineg).
set -o pipefail
mkdir -p gpurun_out
L=$PWD/pulsarfeatureextractor_amd/lib
export PYTHONUNBUFFERED=1
PFE_LIBRARY=$L/libpfe_pre.so timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_a.npz > gpurun_out/ab_dump.log 2>&1 &&
timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_b.npz >> gpurun_out/ab_dump.log 2>&1 &&
PFE_LIBRARY=$L/libpfe_sin2.so timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_c.npz >> gpurun_out/ab_dump.log 2>&1 &&
python tools/lib_outputs.py compare gpurun_out/out_a.npz gpurun_out/out_b.npz > gpurun_out/ab_compare.txt 2>&1; tail -1 gpurun_out/ab_compare.txt
python tools/lib_outputs.py compare gpurun_out/out_a.npz gpurun_out/out_c.npz > gpurun_out/ab_compare_c.txt 2>&1; tail -1 gpurun_out/ab_compare_c.txt
for r in 1 2; do
  for lib in libpfe_pre.so libpfe.so libpfe_sin2.so; do
    PFE_LIBRARY=$L/$lib timeout -k 10 200 python bench.py --path bates22 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_s.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab_s.json').readlines()[-1]);print('$lib',round(d['value']),round(d['ms_per_step'],1))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sin_prof -o trace -- python3 bench.py --path bates22 --steps 2 --warmup 1 --no-cpu-baseline --option serial=1 > /dev/null 2>&1
grep -h sineg gpurun_out/sin_prof/trace_kernel_stats.csv | cut -d, -f1-4
