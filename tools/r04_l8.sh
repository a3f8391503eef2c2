# round 4 (temporary driver): PFD part-reduction width A/B (E = 8 vs 12), pfd22 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in "" e12; do
    PFE_LIBRARY=pulsarfeatureextractor_amd/lib/libpfe${v:+_$v}.so timeout -k 10 300 python3 bench.py --path pfd \
      --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04_pfd_e${v:-8}_$r.json 2> gpurun_out/r04_pfd_e.err || exit 1
  done
done
timeout -k 10 600 python3 bench.py --path pfd22 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04_pfd22.json 2> gpurun_out/r04_pfd22.err
