#!/bin/bash
# Phase cycles (instrumented library) of the 22-score chain, the PFD solve statistics for the
# frozen PFD operation count, two SQ counter passes of the 22-score chain (product library,
# serialised groups), and the PFD 22-score bench line.
set -e
set -o pipefail
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lm_profile.py --n 262144 > gpurun_out/r03_lm_phases.json 2> gpurun_out/r03_lm_phases.err || { tail -20 gpurun_out/r03_lm_phases.err; exit 1; }
echo phases-done
timeout -k 10 300 python -u tools/lm_profile.py --path pfd22 --solver batched --n 1024 > gpurun_out/r03_lmprof_pfd22.json 2> gpurun_out/r03_lmprof_pfd22.err || { tail -20 gpurun_out/r03_lmprof_pfd22.err; exit 1; }
echo pfd-stats-done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA"
i=0
for p in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d gpurun_out/r03_sq/p$i -o pmc -- \
    python3 bench.py --path bates22 --n 262144 --steps 2 --warmup 1 --no-cpu-baseline --option serial=1 > gpurun_out/r03_sq_p$i.log 2>&1
  echo "sq pass $i done"
done
python3 tools/sq_summary.py gpurun_out/r03_sq/p1 gpurun_out/r03_sq/p2 > gpurun_out/r03_sq_summary.json
echo sq-done
timeout -k 10 300 python3 bench.py --path pfd22 --steps 3 --warmup 1 > gpurun_out/r03_bench_pfd22.json 2> gpurun_out/r03_bench_pfd22.err || { tail -20 gpurun_out/r03_bench_pfd22.err; exit 1; }
echo pfd22-bench-done
# config 5 at N > 1: 2 gloo ranks sharing the box's one GPU (RCCL refuses two ranks per device)
PFE_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 5 --warmup 1 --config5-n 1000000 > gpurun_out/r03_rehearse_2rank_gloo.json 2> gpurun_out/r03_rehearse_2rank_gloo.err || { tail -30 gpurun_out/r03_rehearse_2rank_gloo.err; exit 1; }
echo rehearsal-done
