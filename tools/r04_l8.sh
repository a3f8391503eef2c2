# round 4 (temporary driver): Bates 4-parameter pooled kernels at 3 waves/SIMD (28 slots) A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in "" g1 g2; do
    PFE_LIBRARY=pulsarfeatureextractor_amd/lib/libpfe${v:+_$v}.so timeout -k 10 300 python3 bench.py --path bates22 \
      --n 1000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04_b22_${v:-base}_$r.json 2> gpurun_out/r04_b22.err || exit 1
  done
done
