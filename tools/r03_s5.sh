#!/bin/bash
# golden-set GPU dumps of three builds (uncontracted, FMA, FMA + reciprocal quotients) for the
# host-side envelope reports
set -o pipefail
mkdir -p gpurun_out
for L in nofma fma0; do
  PFE_LIBRARY=pulsarfeatureextractor_amd/lib/libpfe_$L.so timeout -k 10 200 python -u tools/golden_dump.py gpurun_out/r03_golden_$L.npz > gpurun_out/r03_dump_$L.log 2>&1 || { tail -20 gpurun_out/r03_dump_$L.log; exit 1; }
done
timeout -k 10 200 python -u tools/golden_dump.py gpurun_out/r03_golden_rcp.npz > gpurun_out/r03_dump_rcp.log 2>&1 || { tail -20 gpurun_out/r03_dump_rcp.log; exit 1; }
ls -la gpurun_out/*.npz
