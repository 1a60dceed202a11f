set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frame_rms.py tests/test_gpu_parity.py tests/test_gpu_edge_inputs.py > gpurun_out/g4_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/g4_tests.txt; [ $rc = 0 ] || exit $rc
SDSP_LIB_PATH=$GRAFT_REPO_ROOT/stratum-dsp_amd/lib_exp/lib_s23.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stft.py > gpurun_out/g4_stft_s23.txt 2>&1; rc=$?; tail -2 gpurun_out/g4_stft_s23.txt; [ $rc = 0 ] || exit $rc
bash tools/kernel_ab.sh rms "k_frame_rms_run|k_peak_abs" base rms0 base rms0
SDSP_PROBE_SIZES=2048 SDSP_PROBE_ROUNDS=3 timeout -k 10 300 python3 -u tools/stft_probe.py stratum-dsp_amd/lib/libstratum_hip.so stratum-dsp_amd/lib_exp/lib_s2.so stratum-dsp_amd/lib_exp/lib_s3.so stratum-dsp_amd/lib_exp/lib_s23.so | tee gpurun_out/g4_stft2048_ab.jsonl
