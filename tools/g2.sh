set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_key_energy.py > gpurun_out/g2_tests.txt 2>&1; rc=$?; tail -5 gpurun_out/g2_tests.txt; grep -E "rigorous certificate|key-energy fields" gpurun_out/g2_tests.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python3 -u tools/key_scale_check.py --n 1024 --sets config2 --out gpurun_out/g2_keyscale.jsonl > gpurun_out/g2_keyscale.log 2>&1; echo "keyscale rc=$?"; tail -2 gpurun_out/g2_keyscale.log | cut -c1-600
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/g2_bench.json 2> gpurun_out/g2_bench.err; echo "bench rc=$?"; python3 -c "
import json,re;l=open('gpurun_out/g2_bench.json').read().strip().splitlines()[-1];d=json.loads(l);print(d['value'],d['ms_per_step'],d.get('sclk_mhz_timed'));print(re.findall(r'.{0,30}rerun.{0,40}',l))"
