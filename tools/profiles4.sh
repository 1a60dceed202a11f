#!/bin/bash
# Regenerates the round's committed profiles (run on the GPU box from the repo root):
#   bash tools/profiles4.sh <tag>        then copy gpurun_out/prof_<tag>/ files into profiles/
set -o pipefail
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 $R/bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/conc -o $tag -- python3 $R/bench.py --tracks 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > $O/conc.json 2> $O/conc.err &&
python3 $R/tools/kdur.py $O/conc/${tag}_kernel_trace.csv 3000 > $O/conc_kdur.txt &&
SDSP_SERIAL_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o $tag -- python3 $R/bench.py --tracks 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > $O/serial.json 2> $O/serial.err &&
python3 $R/tools/step_kernels.py $O/serial/${tag}_kernel_trace.csv 4 > $O/serial_step.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe -o $tag -- python3 $R/tools/stft_probe.py > $O/probe.jsonl 2> $O/probe.err &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_stft --output-format csv -d $O/fetch -o $tag -- python3 $R/bench.py --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline --no-probe > $O/fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_stft --output-format csv -d $O/write -o $tag -- python3 $R/bench.py --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline --no-probe > $O/write.log 2>&1 &&
python3 $R/tools/pmc_stft.py 8192 $O/fetch/${tag}_counter_collection.csv $O/write/${tag}_counter_collection.csv $O/fetch.log > $O/pmc_stft8192.json &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_stft --output-format csv -d $O/fetch2 -o $tag -- python3 $R/bench.py --workload bpm-only --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline --no-probe > $O/fetch2.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_stft --output-format csv -d $O/write2 -o $tag -- python3 $R/bench.py --workload bpm-only --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline --no-probe > $O/write2.log 2>&1 &&
python3 $R/tools/pmc_stft.py 2048 $O/fetch2/${tag}_counter_collection.csv $O/write2/${tag}_counter_collection.csv $O/fetch2.log > $O/pmc_stft2048.json &&
echo "profiles done" && cat $O/serial_step.txt | head -12 && head -12 $O/conc_kdur.txt
