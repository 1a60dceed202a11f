set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g10_smoke.txt 2>&1; rc=$?; tail -3 gpurun_out/g10_smoke.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/g10_bench20.json 2> gpurun_out/g10_bench20.err; rc=$?; echo "bench rc=$rc"; [ $rc = 0 ] || exit $rc
python3 -c "
import json;d=json.loads(open('gpurun_out/g10_bench20.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['sclk_mhz_timed']['median'],d['roofline']['frac'],d['roofline']['isolated']['ms_per_track'],d['key_reruns_last_step'],d['parity_sample'])"
