set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in; do
SDSP_LIB_PATH=$GRAFT_REPO_ROOT/stratum-dsp_amd/lib_exp/lib_$v.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_key_energy.py -k "bitexact or near_decision" > gpurun_out/g15_tests_$v.txt 2>&1; rc=$?; tail -2 gpurun_out/g15_tests_$v.txt; [ $rc = 0 ] || exit $rc
done
bash tools/kernel_ab.sh kfold2 k_mask_rp base f2 base f2 base f2 base f2 base f2
