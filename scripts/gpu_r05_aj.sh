# Round 5: (1) k_acnet with the policy GEMM skipped (skip4) and with the dense + policy GEMMs skipped (skip6), A/B only;
# (2) the few-env stepper with the step's views precomputed per launch (FewStepCtx; build/libmagent_fewctx.so) against
# the product build: parity of the few-env tests, then 8 / 64 envs alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05aj}
mkdir -p $O
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
MAGENT_LIB=$B/libmagent_fewctx.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "small_e or few_pipe or bigq" > $O/tests_fewctx.log 2>&1 || { tail -30 $O/tests_fewctx.log; exit 1; }
tail -1 $O/tests_fewctx.log
for V in "" _skip4 _skip6 ""; do
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 200 python scripts/bench_policy.py --net acnet > $O/acnet$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/acnet$V.json')); print('acnet$V ms %.3f tflops %.1f frac %.3f' % (d['ms_median'], d['tflops'], d['frac']))"
done
for R in 1 2; do
for V in "" _fewctx; do
for E in 8 64; do
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/b${E}$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b${E}$V.json')); print('rep $R lib$V $E envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'check', d['check']['ok'])"
done
done
done
