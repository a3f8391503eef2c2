#!/bin/bash
# SQ counter passes of the serialised 22-score chain for one or more libpfe builds:
#   tools/r05_sq.sh <tag> <lib> [<lib> ...]     -> gpurun_out/r05_sq_<tag>_<lib>.json
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_IFETCH SQ_INSTS_BRANCH"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"
P3="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VSKIPPED"
for L in "$@"; do
  b=$(basename $L .so)
  i=0
  for p in "$P1" "$P2" "$P3"; do
    i=$((i + 1))
    PFE_LIBRARY=$L timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d gpurun_out/r05_sq_${tag}_$b/p$i -o pmc -- \
      python3 bench.py --path bates22 --n 262144 --steps 2 --warmup 1 --no-cpu-baseline --option serial=1 \
      > gpurun_out/r05_sq_${tag}_${b}_p$i.log 2>&1 || { tail -20 gpurun_out/r05_sq_${tag}_${b}_p$i.log; exit 1; }
  done
  python3 tools/sq_summary.py gpurun_out/r05_sq_${tag}_$b/p1 gpurun_out/r05_sq_${tag}_$b/p2 gpurun_out/r05_sq_${tag}_$b/p3 > gpurun_out/r05_sq_${tag}_$b.json
done
python3 - "$tag" "$@" <<'P'
import json, os, sys
tag = sys.argv[1]
for L in sys.argv[2:]:
    b = os.path.basename(L)[:-3]
    d = json.load(open(f"gpurun_out/r05_sq_{tag}_{b}.json"))
    print("==", b)
    for k, v in d.items():
        if "pfe::k_" not in k or v.get("SQ_INSTS_VALU_per_wave", 0) < 1e5:
            continue
        keys = ["SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_THREAD_CYCLES_VALU", "SQ_INSTS_SALU", "SQ_IFETCH", "SQ_INSTS_BRANCH",
                "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64",
                "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_VSKIPPED"]
        print(k.split("(")[0], " ".join(f"{x[8:] if x.startswith('SQ_INSTS') else x[3:]}={v.get(x + '_per_wave', 0)/1e6:.2f}M" for x in keys),
              f"valu_frac={v.get('frac_SQ_ACTIVE_INST_VALU', 0):.3f} waitinst={v.get('frac_SQ_WAIT_INST_ANY', 0):.3f}")
P
