#!/bin/bash
# Round-2 measurement pass (GPU box, repo root): the default bench line, the kernel trace and
# the two HBM PMC passes of its headline kernel, the serialised 22-score kernel trace and two
# SQ counter passes over the 22-score path.  Each step has its own time limit; stop at the
# first failure.
set -e
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/r02_bench_default.json 2> gpurun_out/r02_bench_default.err
echo bench-done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_prof_trace -o trace -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/r02_prof_trace.log 2>&1
echo trace-done
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r02_prof_fetch -o pmc -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/r02_prof_fetch.log 2>&1
echo fetch-done
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r02_prof_write -o pmc -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/r02_prof_write.log 2>&1
echo write-done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_prof_b22 -o trace -- \
  python3 bench.py --path bates22 --steps 3 --warmup 1 --no-cpu-baseline --option serial=1 > gpurun_out/r02_prof_b22.log 2>&1
echo b22-trace-done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA"
i=0
for p in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d gpurun_out/r02_sq/p$i -o pmc -- \
    python3 bench.py --path bates22 --n 262144 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02_sq_p$i.log 2>&1
  echo "sq pass $i done"
done
python3 tools/sq_summary.py gpurun_out/r02_sq/p1 gpurun_out/r02_sq/p2 > gpurun_out/r02_sq_summary.json
echo measure-done
