set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PFE_LIBRARY=$PWD/abl/libpfe_base.so timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_base.npz > gpurun_out/ab_dump.log 2>&1 &&
PFE_LIBRARY=$PWD/abl/libpfe_rowdiv.so timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_new.npz >> gpurun_out/ab_dump.log 2>&1 &&
python tools/lib_outputs.py compare gpurun_out/out_base.npz gpurun_out/out_new.npz > gpurun_out/ab_compare.txt 2>&1; tail -3 gpurun_out/ab_compare.txt;
bash tools/ab_lib_bates.sh $PWD/abl/libpfe_base.so $PWD/abl/libpfe_rowdiv.so 2>&1 | grep -v amdgpu.ids
