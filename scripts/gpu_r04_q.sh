# Round 4: the engine's automatic steps per launch (rollout_substeps(0), bench default) -- its tests and the pipe at
# 64 steps per launch, then the bench lines it gives at configs[3] shapes, 8192 envs and the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04q}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_rollout_gpu.py::test_rollout_substeps_auto_choice" "tests/test_rollout_gpu.py::test_rollout_few_pipe_matches_queue_step" \
  "tests/test_rollout_gpu.py::test_rollout_small_e_matches_oracle" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for E in 8 64 8192; do
  timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/e$E.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'ms/step %.4f' % d['ms_per_step'], 'S', d['config']['steps_per_launch'], d['check']['ok'])" $O/e$E.json
done
timeout -k 10 300 python bench.py > $O/def.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'ms/step %.4f' % d['ms_per_step'], 'S', d['config']['steps_per_launch'], d['check']['ok'], 'traffic', d['roofline']['traffic'])" $O/def.json
