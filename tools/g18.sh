set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/g18_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/g18_tests.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g18_smoke.txt 2>&1; rc=$?; tail -2 gpurun_out/g18_smoke.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/g18_bench.json 2> gpurun_out/g18_bench.err; rc=$?; echo "bench rc=$rc"; [ $rc = 0 ] || exit $rc
python3 -c "
import json;d=json.loads(open('gpurun_out/g18_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['sclk_mhz_timed']['median'],d['roofline']['frac'],d['roofline']['isolated']['ms_per_track'],d['key_reruns_last_step'],d['parity_sample'])"
