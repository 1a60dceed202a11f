#!/bin/bash
# Regenerates the committed profiles (run on the GPU box from the repo root):
#   bash tools/profiles.sh r01
# then copy gpurun_out/prof_<tag>/ files into profiles/ (see profiles/README.md).
set -o pipefail
tag=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 $R/bench.py > $O/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/conc -o $tag -- python3 $R/bench.py --tracks 1024 --steps 2 --warmup 1 --no-cpu-baseline > $O/conc.log 2>&1 &&
SDSP_SERIAL_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o $tag -- python3 $R/bench.py --tracks 1024 --steps 2 --warmup 1 --no-cpu-baseline > $O/serial.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_stft_mag --kernel-trace --output-format csv -d $O/fetch -o $tag -- python3 $R/bench.py --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_stft_mag --kernel-trace --output-format csv -d $O/write -o $tag -- python3 $R/bench.py --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1
