set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/env_e2e.sh ls 3 "" "SDSP_LAST_SHARE=0.75" "SDSP_LAST_SHARE=0.6"
