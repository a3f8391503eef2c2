#!/bin/bash
# Bit-identity + throughput A/B of two libpfe builds (run on the GPU box from the repo root):
#   tools/ab_libs_exact.sh <libA.so> <libB.so>
# Dumps every 22-score output of both builds (tools/lib_outputs.py), compares them bit for
# bit, then alternates the 22-score bench (tools/ab_lib_bates.sh).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PFE_LIBRARY=$1 timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_a.npz > gpurun_out/ab_dump.log 2>&1 &&
PFE_LIBRARY=$2 timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_b.npz >> gpurun_out/ab_dump.log 2>&1 &&
python tools/lib_outputs.py compare gpurun_out/out_a.npz gpurun_out/out_b.npz > gpurun_out/ab_compare.txt 2>&1
tail -3 gpurun_out/ab_compare.txt
bash tools/ab_lib_bates.sh "$1" "$2" 2>&1 | grep -v amdgpu.ids
