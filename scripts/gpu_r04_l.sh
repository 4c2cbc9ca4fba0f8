# Round 4: the pipelined stepper's workgroup team forms (MFX_FEW_PAR_FORMS): parity, stamps, configs[3] A/B;
# the counter list (instruction-cache counters on gfx950?).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04l}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -i -E "ICACHE|SQC_IC|INST_CACHE" $O/counters.txt | head -20 || true
T="tests/test_rollout_gpu.py::test_rollout_few_pipe_matches_queue_step tests/test_rollout_gpu.py::test_rollout_small_e_matches_oracle"
MFX_FEW_PAR_FORMS=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu $T > $O/tests_par.log 2>&1 || { tail -60 $O/tests_par.log; exit 1; }
grep -E "passed|failed" $O/tests_par.log | tail -1
for V in 0 1; do
  MFX_FEW_PAR_FORMS=$V MAGENT_LIB=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 200 \
      python scripts/stamps_few.py --envs 8 > $O/stamps_p$V.txt 2>&1 || { tail -20 $O/stamps_p$V.txt; exit 1; }
  echo "== par forms $V"; grep -E "pipelined|agents:" $O/stamps_p$V.txt
done
for rep in 1 2; do for V in 0 1; do for E in 8 64; do
  MFX_FEW_PAR_FORMS=$V timeout -k 10 200 python bench.py --total-envs $E --steps 200 --warmup 20 --no-cpu-baseline > $O/e${E}_p$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_p$V.json
done; done; done
