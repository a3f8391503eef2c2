#!/bin/bash
# Round-3 re-check after the squared-norm qrfac and the reader changes: GPU suite + smoke,
# default bench line, serialised 22-score trace, streamed files-to-scores on 50k PHCX files.
set -e
set -o pipefail
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03g_gpu_suite.txt 2>&1 || { tail -60 gpurun_out/r03g_gpu_suite.txt; exit 1; }
tail -3 gpurun_out/r03g_gpu_suite.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03g_smoke.txt 2>&1 || { cat gpurun_out/r03g_smoke.txt; exit 1; }
echo suite-done
timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03g_bench_default.json 2> gpurun_out/r03g_bench_default.err || { tail -30 gpurun_out/r03g_bench_default.err; exit 1; }
echo bench-done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03g_prof_b22 -o trace -- \
  python3 bench.py --path bates22 --steps 3 --warmup 1 --no-cpu-baseline --option serial=1 > gpurun_out/r03g_prof_b22.log 2>&1
echo b22-trace-done
timeout -k 10 600 python -u tools/e2e_bench.py --n 50000 --mode stream --workers 16 --batch 8192 > gpurun_out/r03g_e2e_stream.json 2> gpurun_out/r03g_e2e_stream.err || { tail -30 gpurun_out/r03g_e2e_stream.err; exit 1; }
cat gpurun_out/r03g_e2e_stream.json
