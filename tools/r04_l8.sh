# round 4 (temporary driver): DataBlock kernel variants at nDM = 120
set -o pipefail
cd $GRAFT_REPO_ROOT
run() {  # tag lib opts
  PFE_LIBRARY=pulsarfeatureextractor_amd/lib/$2 timeout -k 10 120 python -u tools/lyon8_long_bench.py \
    --n 1000000 --ld 15360,12800 --steps 10 $3 > gpurun_out/r04v_$1.jsonl 2>&1
}
run base libpfe.so "" && run base_fpm libpfe.so "--opt lyon8_dm=2" && run one libpfe.so "--opt lyon8_dm=3" && \
run one_fpm libpfe.so "--opt lyon8_dm=4" && run w3 libpfe_w3.so "" && run w3_fpm libpfe_w3.so "--opt lyon8_dm=2" && \
run np libpfe_np.so "" && run np_fpm libpfe_np.so "--opt lyon8_dm=2" && run w3np libpfe_w3np.so "" && \
run w3np_fpm libpfe_w3np.so "--opt lyon8_dm=2"
