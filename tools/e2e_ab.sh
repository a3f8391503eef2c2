# streamed-path A/B on one box: plain batches vs ramped ends, alternating (tools/e2e_bench.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  TAG=r04ab${r}p E2E_DEPTH=2 E2E_OPT="--ramp 0" bash tools/gpu_steps.sh e2e || exit 1
  TAG=r04ab${r}r E2E_DEPTH=2 E2E_OPT="--ramp 1" bash tools/gpu_steps.sh e2e || exit 1
done
