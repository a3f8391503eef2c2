#!/bin/bash
# timing probe: the 22-score chain without qrfac's column swaps (libpfe_noswap.so, wrong
# results, timing only) against the product library, serialised trace of each
# (the PFE_PROBE_NO_PIVOT_SWAP hook in lm_group.h was removed after the probe; re-add
# "kmax = j;" before the exchange and build variant noswap with that define to repeat it)
set -e
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/pulsarfeatureextractor_amd/lib
bash tools/ab_lib_bates.sh $L/libpfe.so $L/libpfe_noswap.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03_probe_noswap.txt
PFE_LIBRARY=$L/libpfe_noswap.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_prof_noswap -o trace -- \
  python3 bench.py --path bates22 --steps 2 --warmup 1 --no-cpu-baseline --option serial=1 > gpurun_out/r03_prof_noswap.log 2>&1
echo done
