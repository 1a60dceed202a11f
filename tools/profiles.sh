#!/bin/bash
# Regenerates the committed profiles (run on the GPU box from the repo root):
#   bash tools/profiles.sh r02
# then copy gpurun_out/prof_<tag>/ files into profiles/ (see profiles/README.md).
set -o pipefail
tag=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 $R/bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 600 python3 $R/bench.py > $O/bench2.json 2> $O/bench2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/conc -o $tag -- python3 $R/bench.py --tracks 1024 --steps 2 --warmup 1 --no-cpu-baseline > $O/conc.json 2> $O/conc.err &&
SDSP_SERIAL_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o $tag -- python3 $R/bench.py --tracks 1024 --steps 2 --warmup 1 --no-cpu-baseline > $O/serial.json 2> $O/serial.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe -o $tag -- python3 $R/tools/stft_probe.py > $O/probe.jsonl 2> $O/probe.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_stft --kernel-trace --output-format csv -d $O/fetch -o $tag -- python3 $R/bench.py --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_stft --kernel-trace --output-format csv -d $O/write -o $tag -- python3 $R/bench.py --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_stft --kernel-trace --output-format csv -d $O/sq -o $tag -- python3 $R/bench.py --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline > $O/sq.log 2>&1 &&
python3 $R/tools/kstats.py $O/serial/${tag}_kernel_stats.csv 30 > $O/serial_top.txt &&
python3 $R/tools/timeline.py $O/conc/${tag}_kernel_trace.csv 3000 > $O/conc_timeline.txt &&
python3 $R/tools/streams.py $O/conc/${tag}_kernel_trace.csv 3000 >> $O/conc_timeline.txt &&
python3 $R/tools/pmc_stft.py 8192 $O/fetch/${tag}_counter_collection.csv $O/write/${tag}_counter_collection.csv $O/fetch.log > $O/pmc_stft8192.json &&
timeout -k 10 300 python3 $R/bench.py --tracks 64 --steps 1 --warmup 0 --cpu-tracks 32 --cpu-1thread-tracks 32 > $O/cpu1.json 2> $O/cpu1.err &&
timeout -k 10 500 bash $R/tools/pmc_stft_sq.sh $tag > $O/sq_isolated.txt 2>&1 &&
echo "profiles done"
