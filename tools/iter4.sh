#!/bin/bash
# One build -> measure iteration on the GPU box (from the repo root via gpurun):
#   bash tools/iter4.sh <tag> [pytest files...]
# 1. the given GPU tests (default: STFT + end-to-end parity); 2. a serial-stream kernel trace of a
# 1024-track bench (isolated per-kernel times, tools/kstats.py); 3. a two-stream kernel trace of
# the same bench (per-queue launch durations on the shared chip, tools/kdur.py); 4. the default
# bench line (no CPU baseline).
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
tests=${@:-tests/test_gpu_stft.py tests/test_gpu_parity.py}
timeout -k 10 500 python -u -m pytest $tests -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
SDSP_SERIAL_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o s -- python3 $R/bench.py --tracks 1024 --steps 2 --warmup 1 --no-cpu-baseline > $O/serial.json 2> $O/serial.err || { echo "serial prof failed"; tail -20 $O/serial.err; exit 1; }
python3 $R/tools/kstats.py $O/serial/s_kernel_stats.csv 25 > $O/serial_kstats.txt 2>&1; head -25 $O/serial_kstats.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/conc -o c -- python3 $R/bench.py --tracks 1024 --steps 2 --warmup 1 --no-cpu-baseline > $O/conc.json 2> $O/conc.err || { echo "conc trace failed"; tail -20 $O/conc.err; exit 1; }
python3 $R/tools/kdur.py $O/conc/c_kernel_trace.csv 3000 > $O/conc_kdur.txt 2>&1; head -24 $O/conc_kdur.txt
timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$O/bench.json')); r=d['roofline']; print('bench', d['value'], 'frac', r['frac'], 'ms/launch', r['ms_per_launch'], 'isolated', r.get('isolated'), d['step_ms'])"
