set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u tools/key_scale_check.py --n 1024 --sets config2 --out gpurun_out/g19_keyscale.jsonl > gpurun_out/g19_keyscale.log 2>&1; rc=$?; echo "keyscale rc=$rc"; tail -1 gpurun_out/g19_keyscale.log | cut -c1-600; [ $rc = 0 ] || exit $rc
