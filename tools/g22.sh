set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/kernel_ab.sh kmw 'k_mask_rp' base mw5 mw6 base mw5 mw6 base mw5 mw6
