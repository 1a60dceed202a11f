#!/bin/bash
# One build -> measure iteration on the GPU box (run from the repo root via gpurun):
#   bash tools/iter.sh <tag> [pytest files...]
# 1. the given GPU tests (default: STFT + end-to-end parity), 2. a serial-stream rocprofv3 kernel
# trace of a 512-track bench (isolated per-kernel times), 3. the default two-stream bench line.
set -o pipefail
tag=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$tag
mkdir -p $O
tests=${@:-tests/test_gpu_stft.py tests/test_gpu_parity.py}
timeout -k 10 400 python -u -m pytest $tests -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
SDSP_SERIAL_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o s -- python3 $R/bench.py --tracks 512 --steps 2 --warmup 1 --no-cpu-baseline > $O/serial.json 2> $O/serial.err || { echo "serial prof failed"; tail -20 $O/serial.err; exit 1; }
python3 $R/tools/kstats.py $O/serial/s_kernel_stats.csv 25 > $O/serial_kstats.txt 2>&1; head -25 $O/serial_kstats.txt
timeout -k 10 300 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$O/bench.json')); print('bench', d['value'], 'frac', d['roofline']['frac'], 'ms/launch', d['roofline']['ms_per_launch'], d['step_ms'])"
