#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, kernel trace only) on a 64-track bench
# usage: tools/pmc_run.sh tag "kernel regex" "C1 C2 ..." ["C1 C2 ..." ...]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=$1; rx=$2; shift 2
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --kernel-include-regex "$rx" --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${tag}_$i -o run -- python3 $R/bench.py --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_${tag}_$i.log 2>&1 || exit 1
done
