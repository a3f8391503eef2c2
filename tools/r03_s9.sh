#!/bin/bash
# round-3 measurement: the default bench line, rocprof kernel traces (headline Lyon-8 and the
# 22-score chain with its groups serialised), LM phase profiles (instrumented build)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_default.json 2> gpurun_out/r03_bench_default.err || { tail -30 gpurun_out/r03_bench_default.err; exit 1; }
cat gpurun_out/r03_bench_default.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_prof_lyon8 -o trace -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/r03_prof_lyon8.log 2>&1 || { tail -20 gpurun_out/r03_prof_lyon8.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_prof_b22 -o trace -- python3 bench.py --path bates22 --steps 2 --warmup 1 --no-cpu-baseline --option serial=1 > gpurun_out/r03_prof_b22.log 2>&1 || { tail -20 gpurun_out/r03_prof_b22.log; exit 1; }
timeout -k 10 300 python -u tools/lm_profile.py --path bates22 --n 262144 > gpurun_out/r03_lmprof_bates22_pooled.json 2> gpurun_out/r03_lmprof_b22.err || { tail -20 gpurun_out/r03_lmprof_b22.err; exit 1; }
timeout -k 10 300 python -u tools/lm_profile.py --path pfd22 --solver batched --n 4096 > gpurun_out/r03_lmprof_pfd22.json 2> gpurun_out/r03_lmprof_pfd22.err || { tail -20 gpurun_out/r03_lmprof_pfd22.err; exit 1; }
find gpurun_out/r03_prof_lyon8 gpurun_out/r03_prof_b22 -name "*stats*"
