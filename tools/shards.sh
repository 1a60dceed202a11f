#!/bin/bash
# BASELINE config 3 on a one-GPU box: each of the 8 ranks' 1024-track shards (seeds 1024 r ..) run
# alone on device 0 through bench.py --rank-shard, one process per shard, each line with its error
# count, escalation rate and a 16-track oracle parity sample (the 8-GPU curve itself is the
# driver's).  Lines go to gpurun_out/shard_<r>.json.
#   bash tools/shards.sh [first_rank] [last_rank]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
for r in $(seq "${1:-0}" "${2:-7}"); do
  timeout -k 10 240 python3 -u bench.py --rank-shard "$r" --steps 3 --warmup 1 --no-probe --cpu-tracks 16 \
    --cpu-1thread-tracks 1 > "gpurun_out/shard_$r.json" 2> "gpurun_out/shard_$r.err"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['errors'], d.get('escalation_rate'), d['parity_sample'])" \
    "gpurun_out/shard_$r.json" "$r"
done
