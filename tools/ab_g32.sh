set -o pipefail
L=$PWD/pulsarfeatureextractor_amd/lib
bash tools/ab_libs_exact.sh $L/libpfe_base.so $L/libpfe.so &&
PFE_LIBRARY=$L/libpfe_g32.so timeout -k 10 300 python tools/lib_outputs.py dump gpurun_out/out_g32.npz > /dev/null 2>&1 &&
python tools/lib_outputs.py compare gpurun_out/out_b.npz gpurun_out/out_g32.npz > gpurun_out/g32_compare.txt 2>&1;
grep pooled_out gpurun_out/g32_compare.txt;
PFE_LIBRARY=$L/libpfe_g32.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bates22_gpu.py 2>&1 | tail -3 &&
bash tools/ab_lib_bates.sh $L/libpfe.so $L/libpfe_g32.so 2>&1 | grep -v amdgpu.ids
