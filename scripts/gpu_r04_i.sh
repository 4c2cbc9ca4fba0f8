# Round 4: the pipelined few-env stepper on k_rollout's team step (few_env_step) -- few-env parity tests,
# configs[3] shapes pipe off / on, then the stepper's phase stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04i}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --durations=10 --timeout 200 --timeout-method thread -m gpu \
  "tests/test_rollout_gpu.py::test_rollout_few_pipe_matches_queue_step" \
  "tests/test_rollout_gpu.py::test_rollout_small_e_matches_oracle" \
  "tests/test_rollout_gpu.py::test_rollout_lds_step_matches_hbm_step" \
  "tests/test_rollout_gpu.py::test_rollout_matches_oracle" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for rep in 1 2; do for P in 0 1; do for E in 8 64; do
  MFX_FEW_PIPE=$P timeout -k 10 200 python bench.py --total-envs $E --steps 200 --warmup 20 --no-cpu-baseline > $O/e${E}_p$P.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_p$P.json
done; done; done
for e in 8 64; do
  MAGENT_LIB=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 200 \
      python scripts/stamps_few.py --envs $e > $O/stamps_few_$e.txt 2>&1 || { tail -20 $O/stamps_few_$e.txt; exit 1; }
  cat $O/stamps_few_$e.txt
done
