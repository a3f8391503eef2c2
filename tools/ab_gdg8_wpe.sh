#!/bin/bash
# k_gdg8g at 2 waves per SIMD (spilling) vs the product build, then a 2-rank gloo rehearsal
# of the multi-rank bench path (both ranks on the one GPU).
set -o pipefail
mkdir -p gpurun_out
L=$PWD/pulsarfeatureextractor_amd/lib
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for lib in libpfe.so libpfe_w2g16.so libpfe_w2g32.so; do
    PFE_LIBRARY=$L/$lib timeout -k 10 200 python bench.py --path bates22 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_w.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab_w.json').readlines()[-1]);print('$lib',round(d['value']),round(d['ms_per_step'],1))"
  done
done
PFE_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r02_rehearse2.json 2> gpurun_out/r02_rehearse2.err; echo "rehearsal rc=$?"; grep -v amdgpu.ids gpurun_out/r02_rehearse2.json | cut -c1-400
