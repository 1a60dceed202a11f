set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_feature_configs.py tests/test_gpu_key_energy.py tests/test_gpu_multires.py > gpurun_out/g43_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/g43_tests.txt; [ $rc = 0 ] || exit $rc
bash tools/kernel_ab.sh kseq 'k_novelty|k_mel_norm|k_key_vote|k_tempo_select' base prev base prev
