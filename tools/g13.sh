set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SDSP_LIB_PATH=$GRAFT_REPO_ROOT/stratum-dsp_amd/lib_exp/lib_both.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stft.py > gpurun_out/g13_stft_both.txt 2>&1; rc=$?; tail -2 gpurun_out/g13_stft_both.txt; [ $rc = 0 ] || exit $rc
SDSP_PROBE_ROUNDS=3 bash tools/gpu_stft_ab.sh lib_exp/lib_st3.so lib_exp/lib_or2.so lib_exp/lib_both.so
