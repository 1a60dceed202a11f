set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/g5_gpu_tests.txt 2>&1; rc=$?; tail -4 gpurun_out/g5_gpu_tests.txt; [ $rc = 0 ] || exit $rc
bash tools/kernel_ab.sh mask "k_mask_rp" base mask0 base mask0
