# Round 3: the HIP replay row mover, the algo suite through it (replay fixtures, batched rounds, graph
# training), the policy forward in ValueNet.act, then the whole GPU suite and smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03r2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --durations=0 --timeout 280 --timeout-method thread -m gpu tests/test_replay_gpu.py tests/test_algo_gpu.py > $O/tests_algo.log 2>&1 || { tail -60 $O/tests_algo.log; exit 1; }
grep -E "passed|failed" $O/tests_algo.log | tail -1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
