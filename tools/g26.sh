set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/env_e2e.sh td 3 "" "SDSP_TAIL_DEFER=1"
