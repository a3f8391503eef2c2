#!/bin/bash
# End-of-round check (GPU box, repo root): the GPU suite + smoke, the default bench line, and
# the serialised 22-score kernel trace.  Each step has its own time limit; stop at the first
# failure.
set -e
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/r02_gpu_suite.sh
echo suite-done
timeout -k 10 400 python3 bench.py > gpurun_out/r02_bench_final.json 2> gpurun_out/r02_bench_final.err
echo bench-done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_prof_b22f -o trace -- \
  python3 bench.py --path bates22 --steps 3 --warmup 1 --no-cpu-baseline --option serial=1 > gpurun_out/r02_prof_b22f.log 2>&1
echo b22-trace-done
