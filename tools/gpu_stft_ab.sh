#!/bin/bash
# GPU check of an STFT kernel change: the bit-exact STFT tests, then the isolated kernel timing of
# the product library against experimental builds, alternating (tools/stft_probe.py).
#   bash tools/gpu_stft_ab.sh [lib_exp/lib_<name>.so ...]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stft.py > gpurun_out/stft_tests.txt 2>&1 || { tail -30 gpurun_out/stft_tests.txt; exit 1; }
tail -2 gpurun_out/stft_tests.txt
libs="stratum-dsp_amd/lib/libstratum_hip.so"
for l in "$@"; do libs="$libs stratum-dsp_amd/$l"; done
SDSP_PROBE_ROUNDS=${SDSP_PROBE_ROUNDS:-3} timeout -k 10 300 python3 -u tools/stft_probe.py $libs | tee gpurun_out/stft_probe.jsonl
