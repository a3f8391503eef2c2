#!/bin/bash
# Round-2 probe: Lyon-8 burst A/B, the end-to-end (pinned host) Lyon-8 path, and a kernel
# trace of the sub-band (config 4) bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_lyon8.sh 2>&1 | tee gpurun_out/r02_ab_lyon8.txt || exit 1
timeout -k 10 200 python - <<'PY' 2>&1 | tee gpurun_out/r02_e2e.txt
import sys, os, json
sys.path.insert(0, os.getcwd())
import bench, argparse
args = argparse.Namespace(gpus=1, ld=128, option=[])
ctx = bench.Ctx(argparse.Namespace(gpus=1, option=[]))
print(json.dumps(bench.run_e2e(ctx, args, 10_000_000, 128, steps=5)))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sub -o trace -- \
  python3 bench.py --path subband --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_sub.log 2>&1 || exit 1
find gpurun_out/prof_sub -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -8
