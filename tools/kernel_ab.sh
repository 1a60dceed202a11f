#!/bin/bash
# Per-kernel A/B of experimental library builds (serial streams, 256 tracks, one timed step):
#   bash tools/kernel_ab.sh <tag> <kernel-regex> name1 name2 ...   (lib_exp/lib_<name>.so; "base" = product)
set -o pipefail
tag=$1; rx=$2; shift 2
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then unset SDSP_LIB_PATH; else export SDSP_LIB_PATH=$R/stratum-dsp_amd/lib_exp/lib_$v.so; fi
  O=$R/gpurun_out/ab_${tag}_$v
  SDSP_SERIAL_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o s -- python3 $R/bench.py --tracks ${AB_TRACKS:-256} --steps 1 --warmup 1 --no-cpu-baseline > $O.json 2> $O.err || { echo "$v failed"; tail -5 $O.err; exit 1; }
  python3 - "$O/s_kernel_stats.csv" "$rx" "$v" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r['Name']):
        print(f"{sys.argv[3]:12s} {r['Name'][:50]:50s} calls {r['Calls']:>3} avg {float(r['AverageNs'])/1e3:9.1f} us total {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
done
