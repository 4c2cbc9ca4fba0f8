# Round 5: the few-env stepper's LDS pointers rebuilt on the dynamic LDS base after they come out of the per-launch
# contexts (FLAT -> DS instructions, rollout_big.inc lds_rebase): parity of the few-env / bigq tests on the variant,
# then product vs variant on 8 / 64 envs.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05ap}
mkdir -p $O
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
MAGENT_LIB=$B/libmagent_wave.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "small_e or few_pipe or bigq" > $O/tests_wave.log 2>&1 || { tail -30 $O/tests_wave.log; exit 1; }
tail -1 $O/tests_wave.log
for R in 1 2; do
for V in "" _wave; do
for E in 8 64; do
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/b${E}$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b${E}$V.json')); print('rep $R lib$V $E envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'check', d['check']['ok'])"
done
done
done
