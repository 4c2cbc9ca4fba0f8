set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/all_tests.log 2>&1 || { tail -30 gpurun_out/all_tests.log; exit 1; }
bash scripts/gpu_ab.sh head --steps 60 --warmup 5 > gpurun_out/ab64.txt || exit 1
