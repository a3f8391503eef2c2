#!/bin/bash
# PFD kernel check on the GPU box: parity tests, then dmprof / 22-score throughput (A/B of
# the four-wave dmprof kernel against the single-wave one with the option pfd_waves=1)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pfd_gpu.py tests/test_pfd22_gpu.py tests/test_cli_gpu.py \
  -x -v --timeout 200 --timeout-method thread > gpurun_out/t_pfd.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --path pfd --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pfd4.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --path pfd --steps 5 --warmup 2 --no-cpu-baseline --option pfd_waves=1 > gpurun_out/pfd1.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --path pfd22 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pfd22_4.log 2>&1 || exit 1
echo pfd-check-done
