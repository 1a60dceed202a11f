set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/kernel_ab.sh mk "k_mask_rp" base nobr nn base nobr nn base nobr nn base nobr nn base nobr nn
