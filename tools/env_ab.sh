#!/bin/bash
# Per-kernel A/B of environment switches (serial streams, 256 tracks, one timed step):
#   bash tools/env_ab.sh <tag> <kernel-regex> "" "SDSP_X=1" ...    ("" = default)
set -o pipefail
tag=$1; rx=$2; shift 2
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for ev in "$@"; do
  i=$((i+1))
  O=$R/gpurun_out/envab_${tag}_$i
  env $ev SDSP_SERIAL_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o s -- python3 $R/bench.py --tracks 256 --steps 1 --warmup 1 --no-cpu-baseline > $O.json 2> $O.err || { echo "[$ev] failed"; tail -5 $O.err; exit 1; }
  python3 - "$O/s_kernel_stats.csv" "$rx" "[$ev]" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r['Name']):
        print(f"{sys.argv[3]:24s} {r['Name'][:44]:44s} calls {r['Calls']:>3} avg {float(r['AverageNs'])/1e3:9.1f} us total {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
done
