# Round 5: the reward phase's groups in one pass (their partials' LDS chains overlap; each group summed in the same order,
# one barrier for all groups): the GPU battle + rollout tests on the variant, then product vs variant on 8 / 64 /
# 8192 envs, the 40x40 drop-in, the 64x64 default and 256x256.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05aw}
mkdir -p $O
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
MAGENT_LIB=$B/libmagent_wave.so timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py tests/test_battle_gpu.py > $O/tests_wave.log 2>&1 || { tail -30 $O/tests_wave.log; exit 1; }
tail -1 $O/tests_wave.log
for R in 1 2; do
for V in "" _wave; do
for E in 8 64 8192; do
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/b${E}$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b${E}$V.json')); print('rep $R lib$V $E envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
done
done
done
for V in "" _wave; do
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 200 python scripts/bench_dropin.py --map 40 --agents 128 --seconds 4 --calls > $O/dropin$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/dropin$V.json')); print('lib$V drop-in 40x40 vs ref', '%.3f' % d['hip_vs_ref'], json.dumps(d['us_per_step']['hip_dropin']))"
done
for V in "" _wave; do
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bdef$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bdef$V.json')); print('lib$V default', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 300 python bench.py --map 256 --agents 4096 --steps 20 --warmup 5 --no-cpu-baseline > $O/b256$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b256$V.json')); print('lib$V 256x256', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
done
