set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/lib_ab.sh cert 3 base r5 && bash tools/kernel_ab.sh cert "k_key_vote|k_hpcp_band|k_mask_rp" base r5
