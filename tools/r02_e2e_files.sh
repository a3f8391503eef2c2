#!/bin/bash
# Files -> scores end to end on the GPU box: N synthetic PHCX files, the phase-by-phase
# timing, then the streamed product path (own process) at two batch sizes.
set -e
mkdir -p gpurun_out
N=${N:-50000}
D=/tmp/pfe_e2e_$N
timeout -k 10 600 python3 tools/e2e_bench.py --n $N --dir $D --workers 16 > gpurun_out/r02_e2e_phases.json 2> gpurun_out/r02_e2e_phases.err
cat gpurun_out/r02_e2e_phases.json
for b in 8192 2048; do
  timeout -k 10 300 python3 tools/e2e_bench.py --n $N --dir $D --workers 16 --mode stream --batch $b > gpurun_out/r02_e2e_stream_$b.json 2> gpurun_out/r02_e2e_stream_$b.err
  cat gpurun_out/r02_e2e_stream_$b.json
done
rm -rf $D
