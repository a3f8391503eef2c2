# DataBlock rows of 3-4 numpy chunks (nDM > 128): fp64 moments / 3 waves per SIMD variants
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in "" f4 l3 f4l3; do
  PFE_LIBRARY=pulsarfeatureextractor_amd/lib/libpfe${v:+_$v}.so timeout -k 10 200 python -u tools/lyon8_long_bench.py \
    --n 1000000 --ld 20480,30720,24576 --steps 10 > gpurun_out/r04_dmlong_${v:-base}.jsonl 2>&1 || exit 1
done
