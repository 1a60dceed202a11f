#!/bin/bash
# repeat the serial per-kernel profile N times (new process each) to expose run-to-run variance
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for i in $(seq 1 $1); do
  SDSP_SERIAL_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rep_$i -o run -- python3 $R/bench.py --tracks 256 --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/rep_$i.log 2>&1 || exit 1
done
