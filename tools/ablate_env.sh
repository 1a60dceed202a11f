#!/bin/bash
# kernel-time A/B by environment: tools/ablate_env.sh tag "VAR=val VAR2=val" ...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=$1; shift
i=0
for envs in "$@"; do
  i=$((i+1))
  env_args=$envs
  ( for kv in $env_args; do export "$kv"; done
    SDSP_SERIAL_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/abe_${tag}_$i -o run -- python3 $R/bench.py --tracks 256 --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/abe_${tag}_$i.log 2>&1 ) || exit 1
done
