set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/kernel_ab.sh khe 'k_hpcp_band' base noedel base noedel
