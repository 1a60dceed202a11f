set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_TRACKS=341 bash tools/kernel_ab.sh kv5 'k_key_vote' base prev base prev base prev
