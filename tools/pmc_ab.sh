#!/bin/bash
# One PMC pass per experimental library (64-track bench, kernel-filtered):
#   bash tools/pmc_ab.sh <tag> <kernel-regex> "<counters>" name1 name2 ...   (lib_exp/lib_<name>.so; base = product)
tag=$1; rx=$2; ctr=$3; shift 3
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then unset SDSP_LIB_PATH; else export SDSP_LIB_PATH=$R/stratum-dsp_amd/lib_exp/lib_$v.so; fi
  O=$R/gpurun_out/pmcab_${tag}_$v
  timeout -k 10 200 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --kernel-trace --output-format csv -d $O -o run -- python3 $R/bench.py --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline > $O.log 2>&1 || exit 1
  echo "== $v"; python3 $R/tools/pmc.py $(find $O -name "*counter_collection.csv")
done
