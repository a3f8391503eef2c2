#!/bin/bash
# A/B of one libpfe build under two environments on the 22-score path.
#   tools/ab_env.sh "VAR=a" "VAR=b" [n]
set -e
mkdir -p gpurun_out
N=${3:-100000}
env $1 timeout -k 10 300 python tools/bates_throughput.py --n $N --reps 3 --save gpurun_out/ab_A.npz > gpurun_out/ab_A.json
env $2 timeout -k 10 300 python tools/bates_throughput.py --n $N --reps 3 --save gpurun_out/ab_B.npz > gpurun_out/ab_B.json
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
