# round 4 (temporary driver; tools/gpu_steps.sh holds the named steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r04 bash tools/gpu_steps.sh sq_l8dm && \
TAG=r04 L8LD=15360,30720,9216 bash tools/gpu_steps.sh l8long && \
TAG=r04 bash tools/gpu_steps.sh pytest:tests/test_pfd_gpu.py pfdab && \
TAG=r04old L8LD=15360,12800 L8OPT="--opt lyon8_dm=1" bash tools/gpu_steps.sh l8long && \
TAG=r04fpm L8LD=15360,12800 L8OPT="--opt lyon8_dm=2" bash tools/gpu_steps.sh l8long && \
TAG=r04 bash tools/gpu_steps.sh pytest:tests/test_all30_gpu.py e2e
