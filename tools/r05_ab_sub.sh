#!/bin/bash
# Sub-band kernel A/B (GPU box, repo root):  tools/r05_ab_sub.sh <tag> <libA> <libB> [<libC> ...]
#   1. tests/test_subband_gpu.py on the default library
#   2. every library output of each B, C, ... against A (tools/lib_outputs.py), bit for bit
#   3. config 4 (bench.py --path subband) over all libraries in turn, three rounds
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
tag=$1; shift
A=$1; shift
L=$PWD/pulsarfeatureextractor_amd/lib
O=gpurun_out/r05_ab_$tag.txt
mkdir -p gpurun_out
TAG=r05 bash tools/gpu_steps.sh pytest:tests/test_subband_gpu.py || exit 1
PFE_LIBRARY=$L/$A timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/sub_a.npz > gpurun_out/ab_sub_dump.log 2>&1 ||
  { tail -20 gpurun_out/ab_sub_dump.log; exit 1; }
: > $O
for B in "$@"; do
  PFE_LIBRARY=$L/$B timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/sub_b.npz >> gpurun_out/ab_sub_dump.log 2>&1 ||
    { tail -20 gpurun_out/ab_sub_dump.log; exit 1; }
  python tools/lib_outputs.py compare gpurun_out/sub_a.npz gpurun_out/sub_b.npz > gpurun_out/ab_sub_compare.txt 2>&1
  { echo "== outputs A=$A vs $B"; grep -i "sub" gpurun_out/ab_sub_compare.txt; tail -1 gpurun_out/ab_sub_compare.txt; } >> $O
done
echo "== config 4 (16 x 256, 1M candidates), libraries in turn" >> $O
for r in 1 2 3; do
  for lib in $A "$@"; do
    PFE_LIBRARY=$L/$lib timeout -k 10 120 python bench.py --path subband --steps 20 --warmup 3 --no-cpu-baseline --no-extra \
      > gpurun_out/ab_sub.json 2> gpurun_out/ab_sub.err || { tail -20 gpurun_out/ab_sub.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab_sub.json').readlines()[-1]);r=d['roofline'];print('$lib',round(d['value']/1e6,2),'M cand/s kernel',round(r['avg_kernel_ms'],4),'ms frac',round(r['frac'],4))" >> $O
  done
done
cat $O
