# Round 3: can_absorb parity (HIP vs the reference build) and the whole GPU suite after the view-stream
# and absorption changes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03abs
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_absorb.py > $O/tests_absorb.log 2>&1 || { tail -40 $O/tests_absorb.log; exit 1; }
grep -E "passed|failed" $O/tests_absorb.log | tail -1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
