set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profiles4.sh r06a
