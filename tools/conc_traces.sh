#!/bin/bash
# Two-stream kernel traces of N bench processes (to catch both clock/phase states), each
# summarised by tools/overlap.py:  bash tools/conc_traces.sh <tag> [N]
set -o pipefail
tag=$1; n=${2:-3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for i in $(seq 1 $n); do
  O=$R/gpurun_out/conc_${tag}_$i
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o t -- python3 $R/bench.py --tracks 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > $O.json 2> $O.err || { echo "trace $i failed"; tail -3 $O.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O.json') if l.startswith('{')][-1]); print('trace $i', d['value'], d['roofline']['ms_per_launch'])"
  python3 $R/tools/overlap.py $O/t_kernel_trace.csv > $O.overlap.txt && head -8 $O.overlap.txt
done
