#!/bin/bash
# A/B of libpfe builds on the GPU box (repo root); replaces the per-round one-off drivers
# (round 5's tools/r05_*.sh, in git history).  Libraries are paths or names under
# pulsarfeatureextractor_amd/lib; every run has its own time limit and the script stops at
# the first failure.  Results go to gpurun_out/ab_<kind>_<tag>*.
#
#   tools/ab.sh exact   <tag> <libA> <libB>...  every 22-score / sub-band / Lyon output of each
#                                              B against A, bit for bit (tools/lib_outputs.py)
#   tools/ab.sh bates22 <tag> <lib>...          22-score bench (1M resident), libraries in turn,
#                                              ROUNDS (2) rounds; SERIAL=1 serialises the groups
#   tools/ab.sh trace22 <tag> <lib>...          serialised kernel traces of the 22-score chain,
#                                              twice each, per-kernel ms per 1M table
#   tools/ab.sh sq22    <tag> <lib>...          three SQ counter passes of the serialised chain
#   tools/ab.sh subband <tag> <lib>...          config 4 (bench.py --path subband) in turn
#   tools/ab.sh subpmc  <tag> <lib>...          one LDS / VALU SQ pass of config 4 per library
#   tools/ab.sh l8      <tag> <lib>...          the headline (config 2), OPT="--option k=v" allowed
#   tools/ab.sh l8long  <tag> <lib>...          DataBlock-row Lyon-8 (LD="15360,4224,...")
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
kind=$1; tag=$2; shift 2
L=$PWD/pulsarfeatureextractor_amd/lib
O=gpurun_out
mkdir -p $O
lib() { case "$1" in /*) echo "$1" ;; *) echo "$L/$1" ;; esac; }
name() { basename "$1" .so; }
die() { echo "ab.sh $kind: $1 failed"; tail -20 "$2" 2>/dev/null; exit 1; }

case "$kind" in
  exact)
    A=$(lib "$1"); shift
    PFE_LIBRARY=$A timeout -k 10 300 python tools/lib_outputs.py dump $O/ab_out_a.npz > $O/ab_dump_$tag.log 2>&1 \
      || die "dump $(name $A)" $O/ab_dump_$tag.log
    for b in "$@"; do
      B=$(lib "$b")
      PFE_LIBRARY=$B timeout -k 10 300 python tools/lib_outputs.py dump $O/ab_out_b.npz >> $O/ab_dump_$tag.log 2>&1 \
        || die "dump $(name $B)" $O/ab_dump_$tag.log
      echo "== outputs $(name $A) vs $(name $B)"
      # (a difference is a result, not a failure of the step: every differing set is listed)
      python tools/lib_outputs.py compare $O/ab_out_a.npz $O/ab_out_b.npz > $O/ab_cmp_$tag.txt 2>&1 || true
      grep -v "differs in 0 rows\|: \[\]$" $O/ab_cmp_$tag.txt | tail -40 || true
    done ;;
  bates22)
    for r in $(seq ${ROUNDS:-2}); do
      for l in "$@"; do
        X=$(lib "$l")
        PFE_LIBRARY=$X timeout -k 10 200 python bench.py --path bates22 --steps 4 --warmup 1 --no-cpu-baseline \
          --option serial=${SERIAL:-0} > $O/ab_b22.json 2> $O/ab_b22.err || die "bench $(name $X)" $O/ab_b22.err
        python -c "import json;d=json.loads(open('$O/ab_b22.json').readlines()[-1]);print('$(name $X)',round(d['value']),round(d['ms_per_step'],1))"
      done
    done ;;
  trace22)
    for r in 1 2; do
      for l in "$@"; do
        X=$(lib "$l"); d=$O/ab_tr_${tag}_$(name $X)_$r
        PFE_LIBRARY=$X timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o tr -- \
          python3 bench.py --path bates22 --steps 3 --warmup 1 --no-cpu-baseline --option serial=1 \
          > $d.log 2>&1 || die "trace $(name $X)" $d.log
      done
    done
    python3 - "$tag" "$@" <<'P'
import csv, glob, os, sys
tag = sys.argv[1]
names = ["k_gdgg", "k_gdg8g", "k_dmfitg", "k_sineg", "k_gt1g", "k_ghistg", "k_gfixg"]
print("lib".ljust(22), " ".join(n.rjust(9) for n in names), "sum".rjust(8))
for L in sys.argv[2:]:
    b = os.path.basename(L)[:-3] if L.endswith(".so") else L
    for r in (1, 2):
        f = glob.glob(f"gpurun_out/ab_tr_{tag}_{b}_{r}/**/*kernel_stats.csv", recursive=True)[0]
        avg = {}
        for row in csv.DictReader(open(f)):
            for n in names:
                if f"pfe::{n}<" in row["Name"]:
                    avg[n] = float(row["AverageNs"]) / 1e6
        print(f"{b}#{r}".ljust(22), " ".join(f"{avg.get(n, 0):9.1f}" for n in names), f"{sum(avg.values()):8.1f}")
P
    ;;
  sq22)
    P1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_IFETCH SQ_INSTS_BRANCH"
    P2="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"
    P3="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"
    for l in "$@"; do
      X=$(lib "$l"); b=$(name $X); i=0
      for p in "$P1" "$P2" "$P3"; do
        i=$((i + 1))
        PFE_LIBRARY=$X timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d $O/ab_sq_${tag}_$b/p$i -o pmc -- \
          python3 bench.py --path bates22 --n ${SQN:-262144} --steps 2 --warmup 1 --no-cpu-baseline --option serial=1 \
          > $O/ab_sq_${tag}_${b}_p$i.log 2>&1 || die "sq $b" $O/ab_sq_${tag}_${b}_p$i.log
      done
      python3 tools/sq_summary.py $O/ab_sq_${tag}_$b/p1 $O/ab_sq_${tag}_$b/p2 $O/ab_sq_${tag}_$b/p3 > $O/ab_sq_${tag}_$b.json
      python3 - $O/ab_sq_${tag}_$b.json <<'P'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if "pfe::k_" in k and v.get("SQ_INSTS_VALU_per_wave", 0) > 1e5:
        print(k.split("(")[0], f"valu/wave={v['SQ_INSTS_VALU_per_wave']/1e6:.2f}M",
              f"valu_frac={v.get('frac_SQ_ACTIVE_INST_VALU', 0):.3f}",
              f"waitinst={v.get('frac_SQ_WAIT_INST_ANY', 0):.3f}", f"waves={v['waves']:.0f}")
P
    done ;;
  subband)
    for r in $(seq ${ROUNDS:-3}); do
      for l in "$@"; do
        X=$(lib "$l")
        PFE_LIBRARY=$X timeout -k 10 120 python bench.py --path subband --steps 20 --warmup 3 --no-cpu-baseline --no-extra \
          > $O/ab_sub.json 2> $O/ab_sub.err || die "subband $(name $X)" $O/ab_sub.err
        python -c "import json;d=json.loads(open('$O/ab_sub.json').readlines()[-1]);r=d['roofline'];print('$(name $X)',round(d['value']/1e6,2),'M cand/s kernel',round(r['avg_kernel_ms'],4),'ms frac',round(r['frac'],4))"
      done
    done ;;
  subpmc)
    P="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
    for l in "$@"; do
      X=$(lib "$l"); b=$(name $X)
      PFE_LIBRARY=$X timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d $O/ab_subpmc_${tag}_$b -o pmc -- \
        python3 bench.py --path subband --steps 2 --warmup 1 --no-cpu-baseline --no-extra \
        > $O/ab_subpmc_${tag}_$b.log 2>&1 || die "subpmc $b" $O/ab_subpmc_${tag}_$b.log
      python3 tools/sq_summary.py $O/ab_subpmc_${tag}_$b > $O/ab_subpmc_${tag}_$b.json
      python3 - $O/ab_subpmc_${tag}_$b.json "$b" <<'P'
import json, sys
for k, v in json.load(open(sys.argv[1])).items():
    if "subband" in k:
        print(sys.argv[2], k.split("(")[0], {n[:-9]: round(x, 1) for n, x in v.items() if n.endswith("_per_wave")})
P
    done ;;
  l8)
    for r in $(seq ${ROUNDS:-3}); do
      for l in "$@"; do
        X=$(lib "$l")
        PFE_LIBRARY=$X timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline $OPT \
          > $O/ab_l8.json 2> $O/ab_l8.err || die "l8 $(name $X)" $O/ab_l8.err
        python3 -c "import json;d=json.loads(open('$O/ab_l8.json').readlines()[-1]);r=d['roofline'];print('$(name $X)', round(d['value']/1e9,3),'G cand/s kernel',round(r['avg_kernel_ms'],4),'ms frac',round(r['frac'],4))"
      done
    done ;;
  l8long)
    for r in $(seq ${ROUNDS:-2}); do
      for l in "$@"; do
        X=$(lib "$l")
        PFE_LIBRARY=$X timeout -k 10 300 python -u tools/lyon8_long_bench.py --n 1000000 --ld ${LD:-15360,4224,3840} $OPT \
          > $O/ab_l8l.jsonl 2>&1 || die "l8long $(name $X)" $O/ab_l8l.jsonl
        python3 -c "
import json
for l in open('$O/ab_l8l.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$(name $X)', d['ld'], round(d['avg_kernel_ms'],4), 'ms', round(d['frac_of_8TBps'],4))"
      done
    done ;;
  *)
    echo "unknown kind $kind"; exit 2 ;;
esac
