#!/bin/bash
# 256-bin pooled path (32-lane groups): exactness at <= 128 bins against the previous build,
# the GPU parity tests of the 22-score paths, and 256-bin throughput (new vs previous build).
set -o pipefail
mkdir -p gpurun_out
L=$PWD/pulsarfeatureextractor_amd/lib
export PYTHONUNBUFFERED=1
PFE_LIBRARY=$L/libpfe_base.so timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_a.npz > gpurun_out/ab_dump.log 2>&1 &&
timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_b.npz >> gpurun_out/ab_dump.log 2>&1 &&
python tools/lib_outputs.py compare gpurun_out/out_a.npz gpurun_out/out_b.npz > gpurun_out/ab_compare.txt 2>&1; tail -1 gpurun_out/ab_compare.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_bates22_gpu.py tests/test_pfd22_gpu.py tests/test_all30_gpu.py > gpurun_out/p256_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/p256_tests.log
for lib in libpfe_base.so libpfe.so; do
  PFE_LIBRARY=$L/$lib timeout -k 10 200 python bench.py --path bates22 --lp 256 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/p256_$lib.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/p256_$lib.json').readlines()[-1]);print('$lib lp=256',round(d['value']),round(d['ms_per_step'],1))"
done
