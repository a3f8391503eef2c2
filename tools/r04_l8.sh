set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lyon8_gpu.py > gpurun_out/r04_l8_tests.txt 2>&1 && \
timeout -k 10 200 python -u tools/lyon8_long_bench.py --n 1000000 --ld 15360,12800,9216 > gpurun_out/r04_l8_bench.jsonl 2>&1 && \
timeout -k 10 200 python -u tools/lyon8_long_bench.py --n 1000000 --ld 15360,12800 --opt lyon8_dm=1 >> gpurun_out/r04_l8_bench.jsonl 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_all30_gpu.py > gpurun_out/r04_all30_tests.txt 2>&1 && \
timeout -k 10 400 python -u tools/e2e_bench.py --mode stream --n 50000 --dir /tmp/pfe_e2e --depth 1,2 > gpurun_out/r04_e2e.json 2> gpurun_out/r04_e2e.err
