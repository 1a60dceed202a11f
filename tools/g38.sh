set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 ./tools/check_div_d0 > gpurun_out/g38_d0.txt 2>&1; rc=$?; tail -3 gpurun_out/g38_d0.txt; exit $rc
