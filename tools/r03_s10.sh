#!/bin/bash
# two 22-score builds alternating (libpfe.so = reciprocal quotients + enorm fast
# path, contracted gtol test, squared norm-loss test; jac = + Gaussian Jacobian columns as
# e0 exp(delta)), golden dumps, then the 22-score parity files on the jac build
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=pulsarfeatureextractor_amd/lib
for r in 1 2; do
  for lib in $L/libpfe.so $L/libpfe_jac.so; do
    PFE_LIBRARY=$lib timeout -k 10 200 python bench.py --path bates22 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ab_lib.json 2>gpurun_out/ab_lib.err || { tail gpurun_out/ab_lib.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab_lib.json').readlines()[-1]);print('$(basename $lib)',round(d['value']),round(d['ms_per_step'],1))" | tee -a gpurun_out/r03_ab_jac.txt
  done
done
timeout -k 10 200 python -u tools/golden_dump.py gpurun_out/r03_golden_rcp3.npz > gpurun_out/r03_dump_rcp3.log 2>&1 || { tail -20 gpurun_out/r03_dump_rcp3.log; exit 1; }
PFE_LIBRARY=$L/libpfe_jac.so timeout -k 10 200 python -u tools/golden_dump.py gpurun_out/r03_golden_jac.npz > gpurun_out/r03_dump_jac.log 2>&1 || { tail -20 gpurun_out/r03_dump_jac.log; exit 1; }
PFE_LIBRARY=$L/libpfe_jac.so PFE_PARITY_LOG=gpurun_out/r03_parity_slack_jac.jsonl timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_bates22_gpu.py tests/test_all30_gpu.py tests/test_pfd22_gpu.py > gpurun_out/r03_gpu_jac.txt 2>&1; echo "jac parity rc=$?"
tail -3 gpurun_out/r03_gpu_jac.txt
