set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export SDSP_LIB_PATH=$GRAFT_REPO_ROOT/stratum-dsp_amd/lib_exp/lib_kvprof.so
timeout -k 10 300 python3 -u tools/kv_prof.py 19 > gpurun_out/g20_kv19.txt 2>&1; rc=$?; grep -c kvprof gpurun_out/g20_kv19.txt; tail -4 gpurun_out/g20_kv19.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/kv_prof.py 256 > gpurun_out/g20_kv256.txt 2>&1; rc=$?; tail -6 gpurun_out/g20_kv256.txt; [ $rc = 0 ] || exit $rc
