set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/kernel_ab.sh khu 'k_hpcp_band' base hu2 hu1 base hu2 hu1 base hu2 hu1
