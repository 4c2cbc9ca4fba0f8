# The queue kernel at the 256x256 bench shape against the pipeline (tests/test_rollout_gpu.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bigq
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "bigq_bench_shape or queue_matches" > gpurun_out/bigq/shape.log 2>&1 || { tail -30 gpurun_out/bigq/shape.log; exit 1; }
tail -4 gpurun_out/bigq/shape.log
