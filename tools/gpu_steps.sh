#!/bin/bash
# One harness for the GPU-box measurement steps (replaces the per-round r0x_*.sh one-offs).
#
#   bash tools/gpu_steps.sh STEP [STEP ...]        (from the repo root on the GPU box)
#
# Every step runs under its own time limit, writes under gpurun_out/${TAG}_<step>*, and the
# harness stops at the first failing step (no GPU work after a fault, abort or timeout).
# TAG defaults to r06.  A/B of library builds: tools/ab.sh.  Steps:
#   suite        pytest -m gpu (whole GPU suite)
#   smoke        __graft_entry__.smoke()
#   bench        bench.py --gpus 1 (the default bench line, all extras)
#   trace_l8     rocprofv3 kernel trace of the headline Lyon-8 kernel (bench.py, no extras)
#   pmc_l8       FETCH_SIZE and WRITE_SIZE passes of the same command (one pass each)
#   trace_b22    rocprofv3 kernel trace of the 22-score chain, groups serialised
#   sq_b22       two SQ counter passes over the 22-score path + tools/sq_summary.py
#   l8long       tools/lyon8_long_bench.py over DataBlock lengths (LDS=... ops via L8OPT)
#   trace_l8dm   kernel trace of the nDM = 120 Lyon-8 kernel (tools/lyon8_long_bench.py)
#   pmc_l8dm     FETCH_SIZE / WRITE_SIZE passes of the nDM = 120 command
#   sq_l8dm      two SQ counter passes over the nDM = 120 kernel + tools/sq_summary.py
#   sq_sub       two SQ counter passes over the config-4 sub-band kernel (bench.py --path subband)
#   trace_sub    kernel trace of bench.py --path subband
#   pmc_sub      FETCH_SIZE and WRITE_SIZE passes of the same command (one pass each)
#   e2e          tools/e2e_bench.py --mode stream on 50 000 synthetic PHCX files
#   golden_dump  the 22 scores of every golden set (tools/golden_dump.py; host: envelope_report)
#   pfdab        bench.py --path pfd with the split pipeline (default) and fused (pfd_split=0)
#   pytest:<f>   one test file, e.g. pytest:tests/test_lyon8_gpu.py
set -o pipefail
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-r06}
O=gpurun_out

fail() { echo "step $1 failed"; tail -40 "$2" 2>/dev/null; exit 1; }

for step in "$@"; do
  case "$step" in
    suite)
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
        > $O/${T}_gpu_suite.txt 2>&1 || fail suite $O/${T}_gpu_suite.txt
      tail -3 $O/${T}_gpu_suite.txt ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.txt 2>&1 \
        || fail smoke $O/${T}_smoke.txt ;;
    bench)
      timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/${T}_bench_default.json \
        2> $O/${T}_bench_default.err || fail bench $O/${T}_bench_default.err ;;
    trace_l8)
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_l8 -o trace -- \
        python3 bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline > $O/${T}_prof_l8.log 2>&1 \
        || fail trace_l8 $O/${T}_prof_l8.log ;;
    pmc_l8)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/${T}_pmc_l8_$c -o pmc -- \
          python3 bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline > $O/${T}_pmc_l8_$c.log 2>&1 \
          || fail pmc_l8 $O/${T}_pmc_l8_$c.log
      done ;;
    trace_b22)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_b22 -o trace -- \
        python3 bench.py --path bates22 --steps 3 --warmup 1 --no-cpu-baseline --option serial=1 \
        > $O/${T}_prof_b22.log 2>&1 || fail trace_b22 $O/${T}_prof_b22.log ;;
    sq_b22)
      P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
      P2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA"
      i=0
      for p in "$P1" "$P2"; do
        i=$((i + 1))
        timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d $O/${T}_sq/p$i -o pmc -- \
          python3 bench.py --path bates22 --n 262144 --steps 2 --warmup 1 --no-cpu-baseline --option serial=1 \
          > $O/${T}_sq_p$i.log 2>&1 || fail sq_b22 $O/${T}_sq_p$i.log
      done
      python3 tools/sq_summary.py $O/${T}_sq/p1 $O/${T}_sq/p2 > $O/${T}_sq_summary.json ;;
    l8long)
      timeout -k 10 300 python -u tools/lyon8_long_bench.py --n 1000000 --ld ${L8LD:-15360,12800,16256,9216} \
        ${L8OPT} > $O/${T}_l8long.jsonl 2>&1 || fail l8long $O/${T}_l8long.jsonl ;;
    trace_l8dm)
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_l8dm -o trace -- \
        python3 tools/lyon8_long_bench.py --n 1000000 --ld 15360 --steps 20 > $O/${T}_prof_l8dm.log 2>&1 \
        || fail trace_l8dm $O/${T}_prof_l8dm.log ;;
    pmc_l8dm)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/${T}_pmc_l8dm_$c -o pmc -- \
          python3 tools/lyon8_long_bench.py --n 1000000 --ld 15360 --steps 5 > $O/${T}_pmc_l8dm_$c.log 2>&1 \
          || fail pmc_l8dm $O/${T}_pmc_l8dm_$c.log
      done ;;
    sq_l8dm)
      P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY"
      P2="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
      i=0
      for p in "$P1" "$P2"; do
        i=$((i + 1))
        timeout -s KILL 180 rocprofv3 --pmc $p --output-format csv -d $O/${T}_sql8dm/p$i -o pmc -- \
          python3 tools/lyon8_long_bench.py --n 1000000 --ld ${L8LD:-15360} --steps 2 ${L8OPT} \
          > $O/${T}_sql8dm_p$i.log 2>&1 || fail sq_l8dm $O/${T}_sql8dm_p$i.log
      done
      python3 tools/sq_summary.py $O/${T}_sql8dm/p1 $O/${T}_sql8dm/p2 > $O/${T}_sql8dm_summary.json ;;
    sq_sub)
      P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY"
      P2="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
      i=0
      for p in "$P1" "$P2"; do
        i=$((i + 1))
        timeout -s KILL 180 rocprofv3 --pmc $p --output-format csv -d $O/${T}_sqsub/p$i -o pmc -- \
          python3 bench.py --path subband --steps 2 --warmup 1 --no-cpu-baseline --no-extra \
          > $O/${T}_sqsub_p$i.log 2>&1 || fail sq_sub $O/${T}_sqsub_p$i.log
      done
      python3 tools/sq_summary.py $O/${T}_sqsub/p1 $O/${T}_sqsub/p2 > $O/${T}_sqsub_summary.json ;;
    trace_sub)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_trsub -o tr -- \
        python3 bench.py --path subband --steps 10 --warmup 2 --no-cpu-baseline --no-extra \
        > $O/${T}_trsub.json 2> $O/${T}_trsub.err || fail trace_sub $O/${T}_trsub.err ;;
    pmc_sub)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/${T}_pmc_sub_$c -o pmc -- \
          python3 bench.py --path subband --steps 5 --warmup 1 --no-cpu-baseline --no-extra \
          > $O/${T}_pmc_sub_$c.log 2>&1 || fail pmc_sub $O/${T}_pmc_sub_$c.log
      done ;;
    e2e)
      timeout -k 10 600 python -u tools/e2e_bench.py --mode stream --n 50000 --dir /tmp/pfe_e2e \
        --depth ${E2E_DEPTH:-1,2} ${E2E_OPT} > $O/${T}_e2e.json 2> $O/${T}_e2e.err || fail e2e $O/${T}_e2e.err ;;
    golden_dump)
      timeout -k 10 300 python -u tools/golden_dump.py $O/${T}_golden_gpu.npz > $O/${T}_golden_dump.log 2>&1 \
        || fail golden_dump $O/${T}_golden_dump.log ;;
    pfdab)
      for v in 1 0; do
        timeout -k 10 300 python3 bench.py --path pfd --steps 10 --warmup 2 --no-cpu-baseline \
          --option pfd_split=$v > $O/${T}_pfd_split$v.json 2> $O/${T}_pfd_split$v.err \
          || fail pfdab $O/${T}_pfd_split$v.err
      done ;;
    pytest:*)
      f=${step#pytest:}
      n=$(basename "$f" .py)
      timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$f" \
        > $O/${T}_${n}.txt 2>&1 || fail "$step" $O/${T}_${n}.txt
      tail -2 $O/${T}_${n}.txt ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step done"
done
