#!/bin/bash
# A/B of two libpfe builds on the 22-score path: throughput + saved outputs for a bitwise diff.
#   tools/ab_bates.sh <libA.so> <libB.so> [n]
set -e
mkdir -p gpurun_out
N=${3:-100000}
timeout -k 10 200 python tools/bates_throughput.py --n $N --reps 3 --lib "$1" --save gpurun_out/ab_A.npz > gpurun_out/ab_A.json
timeout -k 10 200 python tools/bates_throughput.py --n $N --reps 3 --lib "$2" --save gpurun_out/ab_B.npz > gpurun_out/ab_B.json
python - <<'PY'
import json, numpy as np
a = np.load("gpurun_out/ab_A.npz"); b = np.load("gpurun_out/ab_B.npz")
oa, ob = a["out"], b["out"]
same = (oa == ob) | (np.isnan(oa) & np.isnan(ob))
print(json.dumps({"A": json.load(open("gpurun_out/ab_A.json"))["candidates_per_sec"],
                  "B": json.load(open("gpurun_out/ab_B.json"))["candidates_per_sec"],
                  "status_equal": bool((a["status"] == b["status"]).all()),
                  "bitwise_equal_frac_per_score": [round(float(x), 5) for x in same.mean(0)]}))
PY
