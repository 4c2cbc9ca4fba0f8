# Round 4: the pipelined stepper's overlapped filing (MFX_FEW_OVERLAP): parity both ways, stamps and configs[3] A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04k}
mkdir -p $O
export TMPDIR=/tmp
T="tests/test_rollout_gpu.py::test_rollout_few_pipe_matches_queue_step tests/test_rollout_gpu.py::test_rollout_small_e_matches_oracle"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu $T \
  "tests/test_rollout_gpu.py::test_rollout_matches_oracle" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
MFX_FEW_OVERLAP=0 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu $T > $O/tests_ov0.log 2>&1 || { tail -60 $O/tests_ov0.log; exit 1; }
grep -E "passed|failed" $O/tests_ov0.log | tail -1
for V in 0 1; do
  MFX_FEW_OVERLAP=$V MAGENT_LIB=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 200 \
      python scripts/stamps_few.py --envs 8 > $O/stamps_o$V.txt 2>&1 || { tail -20 $O/stamps_o$V.txt; exit 1; }
  echo "== overlap $V"; cat $O/stamps_o$V.txt
done
for rep in 1 2; do for V in 0 1; do for E in 8 64; do
  MFX_FEW_OVERLAP=$V timeout -k 10 200 python bench.py --total-envs $E --steps 200 --warmup 20 --no-cpu-baseline > $O/e${E}_o$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_o$V.json
done; done; done
