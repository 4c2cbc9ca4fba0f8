# Round 5: bigq_file's count store and slot reservation in flight together (one wait instead of two round trips):
# the rollout GPU tests on the variant (queue kernels, few-env, 256x256 bigq), then product vs variant on 8 / 64 envs
# and 256x256 (2048 envs, and 4096 in two chunks).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05ay}
mkdir -p $O
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
MAGENT_LIB=$B/libmagent_wave.so timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py > $O/tests_wave.log 2>&1 || { tail -30 $O/tests_wave.log; exit 1; }
tail -1 $O/tests_wave.log
for R in 1 2; do
for V in "" _wave; do
for E in 8 64; do
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/b${E}$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b${E}$V.json')); print('rep $R lib$V $E envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'check', d['check']['ok'])"
done
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 300 python bench.py --map 256 --agents 4096 --steps 20 --warmup 5 --no-cpu-baseline > $O/b256$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b256$V.json')); print('rep $R lib$V 256x256', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
done
done
