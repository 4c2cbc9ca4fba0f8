# Round 3: the rollout test file with the renumber-mode and LDS-step-mode equivalence tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/modes}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --durations=8 --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
