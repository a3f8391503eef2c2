#!/bin/bash
# two SQ counter passes of the 22-score chain on the final round-3 build (serialised groups)
set -e
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA"
i=0
for p in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d gpurun_out/r03f_sq/p$i -o pmc -- \
    python3 bench.py --path bates22 --n 262144 --steps 2 --warmup 1 --no-cpu-baseline --option serial=1 > gpurun_out/r03f_sq_p$i.log 2>&1
  echo "sq pass $i done"
done
python3 tools/sq_summary.py gpurun_out/r03f_sq/p1 gpurun_out/r03f_sq/p2 > gpurun_out/r03f_sq_summary.json
echo sq-done
