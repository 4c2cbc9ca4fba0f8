set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r03_modes.sh && bash scripts/gpu_r03_qhead.sh
