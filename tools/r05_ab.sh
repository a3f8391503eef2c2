#!/bin/bash
# round-5 A/B driver: parity files first, then alternating bench of two libraries, then a
# serialised kernel trace of the default library.   tools/r05_ab.sh <tag> <libA> <libB> [tests...]
set -o pipefail
export TMPDIR=/tmp
tag=$1; A=$2; B=$3; shift 3
for t in "$@"; do TAG=r05 bash tools/gpu_steps.sh pytest:$t || exit 1; done
bash tools/ab_lib_bates.sh $A $B > gpurun_out/r05_ab_$tag.txt 2>&1 || { cat gpurun_out/r05_ab_$tag.txt; exit 1; }
cat gpurun_out/r05_ab_$tag.txt
TAG=r05_$tag bash tools/gpu_steps.sh trace_b22 || exit 1
cut -d, -f1-4 gpurun_out/r05_${tag}_prof_b22/trace_kernel_stats.csv | grep "pfe::k_" | head -12
