# Round 4: the pipelined few-env form past 64 steps per launch (its lists sized for 1024) -- tests, then configs[3]
# shapes with the engine's choice (the whole timed region as one launch) at K = 256 and 1024.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04r}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_rollout_gpu.py::test_rollout_substeps_auto_choice" "tests/test_rollout_gpu.py::test_rollout_few_pipe_matches_queue_step" \
  "tests/test_rollout_gpu.py::test_rollout_small_e_matches_oracle" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for rep in 1 2; do for K in 256 1024; do for E in 8 64; do
  timeout -k 10 200 python bench.py --total-envs $E --steps $K --warmup 64 --no-cpu-baseline > $O/e${E}_k$K.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'S', d['config']['steps_per_launch'], 'kernel_ms %.3f' % r['kernel_ms'], 'frac %.4f' % r['frac'], d['check']['ok'])" $O/e${E}_k$K.json
done; done; done
