set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/lib_ab.sh tail 3 base t33 t60
