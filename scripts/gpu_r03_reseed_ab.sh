# Round 3: the bigq re-seed regression test against the round-2 re-seed (variant library built with
# -DMFX_AB_R2_RESEED: must FAIL) and the fixed library (must pass); then the new bench-shape replays with
# durations, the default bench (self-check), and the whole GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03r
mkdir -p $O
export TMPDIR=/tmp
L=mean-field-multi-agent-reinforcement-learning_amd/build
MAGENT_LIB=$L/libmagent_r2reseed.so timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k reseed > $O/reseed_r2.log 2>&1
echo "round-2 re-seed variant: pytest exit $?" | tee $O/reseed_r2.status
grep -E "PASSED|FAILED|Error|error [0-9]" $O/reseed_r2.log | head -5
timeout -k 10 400 python -u -m pytest -x -v --durations=0 --timeout 280 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "bench_shape_matches_oracle or reseed" > $O/tests_new.log 2>&1 || { tail -40 $O/tests_new.log; exit 1; }
grep -E "PASSED|FAILED|s call" $O/tests_new.log | head -12
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; cat $O/bench.json; exit 1; }
cat $O/bench.json
timeout -k 10 900 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
