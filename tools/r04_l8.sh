# round 4 (temporary driver): PFD occupancy change, e2e ramp A/B, final suite, smoke, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r04 bash tools/gpu_steps.sh pytest:tests/test_pfd_gpu.py pytest:tests/test_pfd22_gpu.py pfdab && \
TAG=r04nr E2E_OPT=--no-ramp bash tools/gpu_steps.sh e2e && \
TAG=r04 bash tools/gpu_steps.sh e2e suite smoke bench
