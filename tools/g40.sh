set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_key_energy.py -k tail_rerun > gpurun_out/g40_tests.txt 2>&1; rc=$?; tail -5 gpurun_out/g40_tests.txt; exit $rc
