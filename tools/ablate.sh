#!/bin/bash
# kernel-time ablations: per-kernel stats for alternative library builds (serial streams)
# usage: tools/ablate.sh name1 name2 ...   (stratum-dsp_amd/lib_exp/lib_<name>.so; "base" = the normal build)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in "$@"; do
  if [ "$v" = base ]; then unset SDSP_LIB_PATH; else export SDSP_LIB_PATH=$R/stratum-dsp_amd/lib_exp/lib_$v.so; fi
  SDSP_SERIAL_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_$v -o run -- python3 $R/bench.py --tracks 256 --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/ab_$v.log 2>&1 || exit 1
done
