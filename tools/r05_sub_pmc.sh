#!/bin/bash
# One SQ counter pass (LDS conflicts, VALU, waits) of config 4 per library (GPU box, repo root):
#   tools/r05_sub_pmc.sh <tag> <lib> [<lib> ...]   -> gpurun_out/r05_subpmc_<tag>.json
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
L=$PWD/pulsarfeatureextractor_amd/lib
P="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
for lib in "$@"; do
  PFE_LIBRARY=$L/$lib timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d gpurun_out/r05_subpmc_$tag/$lib -o pmc -- \
    python3 bench.py --path subband --steps 2 --warmup 1 --no-cpu-baseline --no-extra \
    > gpurun_out/r05_subpmc_${tag}_$lib.log 2>&1 || { tail -20 gpurun_out/r05_subpmc_${tag}_$lib.log; exit 1; }
done
python3 - "$tag" "$@" <<'PY'
import csv, glob, json, sys
tag, libs = sys.argv[1], sys.argv[2:]
out = {}
for lib in libs:
    f = glob.glob(f"gpurun_out/r05_subpmc_{tag}/{lib}/**/*counter_collection.csv", recursive=True)[0]
    acc, waves = {}, 0.0
    for r in csv.DictReader(open(f)):
        if "subband_fast" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] = acc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    w = acc.get("SQ_WAVES", 1.0)
    out[lib] = {k + "_per_wave": round(v / w, 2) for k, v in acc.items() if k != "SQ_WAVES"}
    out[lib]["waves"] = w
json.dump(out, open(f"gpurun_out/r05_subpmc_{tag}.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
