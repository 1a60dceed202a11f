#!/bin/bash
# Bench bimodality probe (GPU box, repo root): two-stream and serial-stream bench processes
# alternating, rocm-smi sampled while each runs; prints tracks/s with the sampled sclk / power.
#   bash tools/state_probe.sh <tag> [rounds]
set -o pipefail
tag=$1; n=${2:-4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/state_$tag
mkdir -p $O
for i in $(seq 1 $n); do
  for mode in conc serial; do
    ev=""; [ $mode = serial ] && ev="SDSP_SERIAL_STREAMS=1"
    env $ev timeout -k 10 200 python3 $R/bench.py --steps 30 --warmup 1 --no-cpu-baseline --no-probe > $O/${mode}_$i.json 2> $O/${mode}_$i.err &
    pid=$!
    : > $O/${mode}_${i}_smi.txt
    sleep 4
    while kill -0 $pid 2>/dev/null; do
      timeout 10 rocm-smi --showclocks --showpower --showtemp >> $O/${mode}_${i}_smi.txt 2>&1
      sleep 0.5
    done
    wait $pid || { echo "bench $mode $i failed"; tail -3 $O/${mode}_$i.err; exit 1; }
    python3 - $O/${mode}_$i.json $O/${mode}_${i}_smi.txt $mode <<'PY'
import json, sys, re
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
smi = open(sys.argv[2]).read()
sclk = [int(x) for x in re.findall(r"sclk level: \d+: \((\d+)Mhz\)", smi)]
pw = [float(x) for x in re.findall(r"Power \(W\): ([\d.]+)", smi)]
print(f"{sys.argv[3]:6s} {d['value']:8.1f} tracks/s  step median {d['step_ms']['median']:7.1f} ms  sclk samples {sclk}  power {pw}")
PY
  done
done
