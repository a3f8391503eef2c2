#!/bin/bash
# pivoted-basis lmpar (libpfe.so) vs the previous build (libpfe_rcp3.so), alternating; then
# the whole GPU suite and smoke on libpfe.so
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/ab_lib_bates.sh pulsarfeatureextractor_amd/lib/libpfe_rcp3.so pulsarfeatureextractor_amd/lib/libpfe.so > gpurun_out/r03_ab_perm.txt 2>&1 || { cat gpurun_out/r03_ab_perm.txt; tail gpurun_out/ab_lib.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_ab_perm.txt
timeout -k 10 200 python -u tools/golden_dump.py gpurun_out/r03_golden_perm.npz > gpurun_out/r03_dump_perm.log 2>&1 || { tail -20 gpurun_out/r03_dump_perm.log; exit 1; }
bash tools/r03_suite.sh
