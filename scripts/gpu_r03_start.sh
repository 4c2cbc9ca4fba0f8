# Round 3: the GPU tests (new: bench-shape oracle replays at 4 / 16 steps per launch, the bigq re-seed
# regression, the hand-off guard), smoke, and the default bench with its self-check.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "bench_shape_matches_oracle or reseed" > $O/tests_new.log 2>&1 || { tail -40 $O/tests_new.log; exit 1; }
tail -3 $O/tests_new.log
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; cat $O/bench.json; exit 1; }
cat $O/bench.json
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
