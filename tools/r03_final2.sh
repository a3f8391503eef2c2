#!/bin/bash
# End-of-round-3 check (GPU box, repo root): GPU suite + smoke, the default bench line, the
# Lyon-8 headline trace, the Lyon-8 PHCX-shape kernel (lyon8_u8_pow2) trace + HBM PMC passes,
# and the serialised 22-score trace.  Each step has its own limit; stop at the first failure.
set -e
set -o pipefail
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03f_gpu_suite.txt 2>&1 || { tail -60 gpurun_out/r03f_gpu_suite.txt; exit 1; }
tail -3 gpurun_out/r03f_gpu_suite.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03f_smoke.txt 2>&1 || { cat gpurun_out/r03f_smoke.txt; exit 1; }
echo suite-done
timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03f_bench_default.json 2> gpurun_out/r03f_bench_default.err || { tail -30 gpurun_out/r03f_bench_default.err; exit 1; }
echo bench-done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03f_prof_lyon8 -o trace -- \
  python3 bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/r03f_prof_lyon8.log 2>&1
echo lyon8-trace-done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03f_prof_l8p2 -o trace -- \
  python3 tools/lyon8_long_bench.py --ld 16384 --steps 10 > gpurun_out/r03f_prof_l8p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r03f_l8p2_fetch -o pmc -- \
  python3 tools/lyon8_long_bench.py --ld 16384 --steps 3 > gpurun_out/r03f_l8p2_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r03f_l8p2_write -o pmc -- \
  python3 tools/lyon8_long_bench.py --ld 16384 --steps 3 > gpurun_out/r03f_l8p2_write.log 2>&1
echo l8p2-pmc-done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03f_prof_b22 -o trace -- \
  python3 bench.py --path bates22 --steps 3 --warmup 1 --no-cpu-baseline --option serial=1 > gpurun_out/r03f_prof_b22.log 2>&1
echo b22-trace-done
