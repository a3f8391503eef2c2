#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/r03_det.py 5 > gpurun_out/r03_det.txt 2>&1; echo rc=$?
cat gpurun_out/r03_det.txt | grep -v amdgpu.ids
