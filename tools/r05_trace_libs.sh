#!/bin/bash
# Serialised 22-score kernel traces (1M resident candidates) of several libpfe builds, twice
# each, alternating:  tools/r05_trace_libs.sh <tag> <lib> [<lib> ...]
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
for r in 1 2; do
  for L in "$@"; do
    b=$(basename $L .so)
    d=gpurun_out/r05_tr_${tag}_${b}_$r
    PFE_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o tr -- \
      python3 bench.py --path bates22 --steps 3 --warmup 1 --no-cpu-baseline --option serial=1 \
      > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  done
done
python3 - "$tag" "$@" <<'P'
import csv, glob, os, sys
tag = sys.argv[1]
names = ["k_gdgg", "k_gdg8g", "k_dmfitg", "k_sineg", "k_gt1g", "k_ghistg", "k_gfixg"]
print("lib".ljust(22), " ".join(n.rjust(9) for n in names), "sum".rjust(8))
for L in sys.argv[2:]:
    b = os.path.basename(L)[:-3]
    for r in (1, 2):
        f = glob.glob(f"gpurun_out/r05_tr_{tag}_{b}_{r}/**/*kernel_stats.csv", recursive=True)[0]
        avg = {}
        for row in csv.DictReader(open(f)):
            for n in names:
                if f"pfe::{n}<" in row["Name"]:
                    avg[n] = float(row["AverageNs"]) / 1e6
        print(f"{b}#{r}".ljust(22), " ".join(f"{avg.get(n, 0):9.1f}" for n in names), f"{sum(avg.values()):8.1f}")
P
