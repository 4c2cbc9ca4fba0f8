set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r03_qnet_vec.sh && bash scripts/gpu_r03_sub256.sh
