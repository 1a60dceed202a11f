#!/bin/bash
# End-to-end A/B of environment switches (two-stream bench, 1024 x 3-min tracks):
#   bash tools/bench_ab.sh <tag> "" "SDSP_X=1" "SDSP_X=1 SDSP_Y=1" ...    ("" = default)
# One bench process per setting; prints tracks/s, step spread and the in-pipeline 8192 STFT frac.
set -o pipefail
tag=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
i=0
for ev in "$@"; do
  i=$((i+1))
  O=$R/gpurun_out/benchab_${tag}_$i
  env $ev timeout -k 10 240 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe > $O.json 2> $O.err || { echo "[$ev] failed"; tail -5 $O.err; exit 1; }
  python3 - "$O.json" "[$ev]" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print(f"{sys.argv[2]:40s} {d['value']:9.1f} tracks/s  steps {d['step_ms']['all']}  stft8192 {r['ms_per_launch']:7.2f} ms/launch frac {r['frac']:.3f}  stages {d['stage_ms_last_step']}")
PY
done
