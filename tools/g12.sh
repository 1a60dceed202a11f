set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_key_energy.py tests/test_gpu_key_options.py tests/test_gpu_chroma_options.py tests/test_gpu_frame_size.py tests/test_gpu_parity.py tests/test_gpu_edge_inputs.py tests/test_gpu_batch_paths.py > gpurun_out/g12_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/g12_tests.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python3 -u tools/key_scale_check.py --n 1024 --sets config2 --out gpurun_out/g12_keyscale.jsonl > gpurun_out/g12_keyscale.log 2>&1; echo "keyscale rc=$?"; tail -1 gpurun_out/g12_keyscale.log | cut -c1-420
