# Round 3: the reworked replay mover (one wave per row, loads ahead of stores) -- its parity tests, the
# algo tests that run on it, and the sample benchmark.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03rows
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_replay_gpu.py tests/test_algo_gpu.py > $O/tests_replay.log 2>&1 || { tail -40 $O/tests_replay.log; exit 1; }
grep -E "passed|failed" $O/tests_replay.log | tail -1
timeout -k 10 200 python scripts/bench_replay.py > $O/replay2.json 2> $O/replay.err || { tail -20 $O/replay.err; exit 1; }
cat $O/replay2.json
