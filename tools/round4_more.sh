#!/bin/bash
# Round-4 measurements beside tools/profiles4.sh (GPU box, repo root):  bash tools/round4_more.sh <tag>
# three default bench processes (clock-state spread), BASELINE configs 4 and 5, the key-path /
# feature HBM counters with the HBM ceiling (tools/pmc_key.sh), SQ counters over the isolated
# 8192-point STFT (tools/pmc_stft_sq.sh).
set -o pipefail
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/more_$tag
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err || { echo "bench $i failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$i.json')); print('bench', d['value'], d['roofline']['ms_per_launch'])"
done
timeout -k 10 300 python3 $R/bench.py --workload mixed --steps 3 --warmup 1 --no-cpu-baseline --no-probe > $O/config4.json 2> $O/config4.err &&
timeout -k 10 300 python3 $R/bench.py --workload bpm-only --steps 3 --warmup 1 --no-cpu-baseline > $O/config5.json 2> $O/config5.err &&
python3 -c "import json; [print(f, json.load(open('$O/'+f))['value']) for f in ('config4.json','config5.json')]" &&
bash $R/tools/pmc_key.sh $tag &&
SDSP_PROBE_SIZES=8192 bash $R/tools/pmc_stft_sq.sh $tag
