# round 4 (temporary driver): final measurements of the round
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r04 bash tools/gpu_steps.sh e2e golden_dump suite smoke bench
