# round 4 (temporary driver): DataBlock kernel options at nDM = 120
set -o pipefail
cd $GRAFT_REPO_ROOT
run() {  # tag opts
  timeout -k 10 120 python -u tools/lyon8_long_bench.py --n 1000000 --ld 15360,12800,16256 --steps 10 $2 \
    > gpurun_out/r04v_$1.jsonl 2>&1
}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lyon8_gpu.py \
  -k "options_agree or multibatch or golden_dmplane" > gpurun_out/r04v_tests.txt 2>&1 && \
run tab "--opt lyon8_dm=5" && run one_fpm "--opt lyon8_dm=4" && run one "--opt lyon8_dm=3"
