set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_batch_paths.py -k config3 > gpurun_out/g1_config3.txt 2>&1; echo "config3 rc=$?"; tail -3 gpurun_out/g1_config3.txt
SDSP_PROBE_ROUNDS=3 bash tools/gpu_stft_ab.sh lib_exp/lib_asm3.so lib_exp/lib_wksg.so lib_exp/lib_asm3wksg.so
