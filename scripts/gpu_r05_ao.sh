# Round 5: the rush policy's centre test as 2x < W (exact) -- product vs variant on 8 / 64 / 131072 envs -- and the
# phase stamps with the stamp pointer in constant memory (a stamp no longer waits for the phase's stores).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05ao}
mkdir -p $O
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
MAGENT_LIB=$B/libmagent_wave.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "small_e or few_pipe or reference or oracle" > $O/tests_wave.log 2>&1 || { tail -30 $O/tests_wave.log; exit 1; }
tail -1 $O/tests_wave.log
for R in 1 2; do
for V in "" _wave; do
for E in 8 64; do
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/b${E}$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b${E}$V.json')); print('rep $R lib$V $E envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'check', d['check']['ok'])"
done
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bdef$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bdef$V.json')); print('rep $R lib$V default', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
done
done
L=$B/libmagent_stamps.so
MAGENT_LIB=$L timeout -k 10 300 python scripts/stamps_few.py --envs 8 --sub 20 --launches 20 --snap > $O/stamps_few.txt 2>&1 || { tail -20 $O/stamps_few.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_few.txt
MAGENT_LIB=$L timeout -k 10 300 python scripts/stamps_battle.py --envs 8192 --steps 4 > $O/stamps8192.txt 2>&1 || { tail -20 $O/stamps8192.txt; exit 1; }
grep -v amdgpu.ids $O/stamps8192.txt
