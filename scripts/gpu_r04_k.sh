# Round 4: the pipelined stepper's wave-team threshold (MFX_FEW_WAVE_MAX): parity at 512, stamps and configs[3] A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04k}
mkdir -p $O
export TMPDIR=/tmp
MFX_FEW_WAVE_MAX=512 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  "tests/test_rollout_gpu.py::test_rollout_few_pipe_matches_queue_step" \
  "tests/test_rollout_gpu.py::test_rollout_small_e_matches_oracle" > $O/tests512.log 2>&1 || { tail -60 $O/tests512.log; exit 1; }
grep -E "passed|failed" $O/tests512.log | tail -1
for W in 64 128 256 512; do
  MFX_FEW_WAVE_MAX=$W MAGENT_LIB=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 200 \
      python scripts/stamps_few.py --envs 8 > $O/stamps_w$W.txt 2>&1 || { tail -20 $O/stamps_w$W.txt; exit 1; }
  echo "== wave max $W"; grep -E "pipelined|agents:" $O/stamps_w$W.txt
done
for rep in 1 2; do for W in 64 128 256 512; do for E in 8 64; do
  MFX_FEW_WAVE_MAX=$W timeout -k 10 200 python bench.py --total-envs $E --steps 200 --warmup 20 --no-cpu-baseline > $O/e${E}_w$W.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_w$W.json
done; done; done
