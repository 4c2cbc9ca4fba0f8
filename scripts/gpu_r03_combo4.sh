set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03f3 bash scripts/gpu_r03_final2.sh && bash scripts/gpu_r03_qvec4.sh
