set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
true
bash tools/kernel_ab.sh kocc k_features base occ2 base occ2
