# round 4 (temporary driver): DataBlock defaults, headline profile, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r04d L8LD=15360,12800,16256,20480,30720,9216 bash tools/gpu_steps.sh pytest:tests/test_lyon8_gpu.py l8long && \
TAG=r04d_one L8LD=20480,30720 L8OPT="--opt lyon8_dm=3" bash tools/gpu_steps.sh l8long && \
TAG=r04 bash tools/gpu_steps.sh trace_l8 pmc_l8 trace_l8dm pmc_l8dm e2e bench
