set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ising_gpu.py -x -q -m gpu > gpurun_out/ising.log 2>&1
