#!/bin/bash
# End-to-end A/B of environment switches, alternating (two-stream bench, 1024 x 3-min tracks):
#   bash tools/env_e2e.sh <tag> <rounds> "" "SDSP_X=1" ...    ("" = default)
set -o pipefail
tag=$1; rounds=$2; shift 2
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for r in $(seq $rounds); do
i=0
for ev in "$@"; do
  i=$((i+1))
  O=$R/gpurun_out/enve2e_${tag}_${i}_$r
  env $ev timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probe > $O.json 2> $O.err || { echo "[$ev] failed"; tail -5 $O.err; exit 1; }
  python3 - "$O.json" "[$ev]" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
st = d["stage_ms_last_step"]
print(f"{sys.argv[2]:22s} {d['value']:8.1f} tracks/s  ms/step {d['ms_per_step']:7.1f}  sclk {d['sclk_mhz_timed']['median']}  reruns {d.get('key_reruns_last_step')}  rerun_ms {st.get('rerun_ms')}", flush=True)
PY
done
done
