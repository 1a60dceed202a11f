set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_key_energy.py tests/test_gpu_key_options.py > gpurun_out/g37_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/g37_tests.txt; [ $rc = 0 ] || exit $rc
bash tools/kernel_ab.sh krg 'k_hpcp_band' base rng base rng base rng
