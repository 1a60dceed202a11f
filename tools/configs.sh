#!/bin/bash
# Bench lines of the BASELINE configs beside the default one (run on the GPU box from the repo
# root):  bash tools/configs.sh r02
#   config 4: mixed 30 s - 10 min batch (full analysis);  config 5: BPM-only stages a1-a19 over
#   4096 escalation-heavy tracks;  plus the 2048-point STFT PMC passes that give bpm-only's
#   roofline.traffic (profiles/pmc_stft2048.json).
# Outputs: gpurun_out/cfg_<tag>/{config4,config5}.json, fetch2048/ write2048/ (+ logs).
set -o pipefail
tag=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/cfg_$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --workload mixed --steps 3 --warmup 1 --no-cpu-baseline > $O/config4.json 2> $O/config4.err &&
timeout -k 10 300 python3 $R/bench.py --workload bpm-only --steps 3 --warmup 1 --no-cpu-baseline > $O/config5.json 2> $O/config5.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_stft --kernel-trace --output-format csv -d $O/fetch2048 -o f -- python3 $R/bench.py --workload bpm-only --tracks 256 --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch2048.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_stft --kernel-trace --output-format csv -d $O/write2048 -o w -- python3 $R/bench.py --workload bpm-only --tracks 256 --steps 1 --warmup 0 --no-cpu-baseline > $O/write2048.log 2>&1 &&
python3 $R/tools/pmc_stft.py 2048 $O/fetch2048/f_counter_collection.csv $O/write2048/w_counter_collection.csv $O/fetch2048.log > $O/pmc_stft2048.json &&
echo "configs done" && cat $O/config4.json $O/config5.json $O/pmc_stft2048.json
