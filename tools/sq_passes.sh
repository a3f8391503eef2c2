#!/bin/bash
# SQ counter passes over one bench.py step (run on the GPU box from the repo root):
#   tools/sq_passes.sh OUTDIR bench-args...
# Each pass is its own rocprofv3 run (at most 8 SQ counters per pass), under its own limit.
set -e
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA"
i=0
for p in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -k 10 240 rocprofv3 --pmc $p --output-format csv -d "$out/p$i" -o pmc -- \
    python3 bench.py "$@" --no-cpu-baseline > "$out/p$i.log" 2>&1
  echo "pass $i done"
done
python3 tools/sq_summary.py "$out/p1" "$out/p2" > "$out/sq_summary.json"
echo sq-done
