#!/bin/bash
# layout experiment: per-kernel stats for several spectrogram row strides (serial streams)
# usage: tools/stride_sweep.sh "S8 S2" ...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for cfg in "$@"; do
  set -- $cfg
  SDSP_UNFUSED_MASK=1 SDSP_STRIDE8=$1 SDSP_STRIDE2=$2 SDSP_SERIAL_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sw2_$1_$2 -o run -- python3 $R/bench.py --tracks 256 --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/sw2_$1_$2.log 2>&1 || exit 1
done
