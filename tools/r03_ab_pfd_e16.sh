#!/bin/bash
# PFD fold reduction with 16 elements per thread (libpfe.so) vs 8 (libpfe_base.so): PFD
# parity tests on the new build, then the alternating dmprof and 22-score bench lines
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=$PWD/pulsarfeatureextractor_amd/lib
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pfd_gpu.py tests/test_pfd22_gpu.py > gpurun_out/r03_pfd_e16_tests.txt 2>&1 || { tail -30 gpurun_out/r03_pfd_e16_tests.txt; exit 1; }
tail -1 gpurun_out/r03_pfd_e16_tests.txt
for r in 1 2; do
  for lib in libpfe_base.so libpfe.so; do
    PFE_LIBRARY=$L/$lib timeout -k 10 200 python bench.py --path pfd --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_pfd.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab_pfd.json').readlines()[-1]);print('$lib pfd',round(d['value']/1e6,3),'M folds/s kernel',round(d['roofline']['avg_kernel_ms'],3),'ms')"
  done
done
