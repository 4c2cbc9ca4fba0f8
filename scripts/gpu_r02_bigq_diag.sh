set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bigq
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "queue_matches" > gpurun_out/bigq/t2.log 2>&1; grep -E "AssertionError: \(|passed|failed" gpurun_out/bigq/t2.log | head -5
