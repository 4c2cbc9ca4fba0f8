# Round 5: where the steps stand after the wave-team and LDS-rebase work: the GPU battle + rollout tests, the drop-in
# against _ref at 40x40, the few-env and 8192-env stamps, and the bench lines 8 / 64 / 8192 / default.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05aq}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py tests/test_battle_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python scripts/bench_dropin.py --map 40 --agents 128 --seconds 4 --calls > $O/dropin_40.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/dropin_40.json')); print('drop-in 40x40 vs ref', '%.3f' % d['hip_vs_ref'], json.dumps(d['us_per_step']['hip_dropin']))"
for E in 8 64 8192; do
timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/b$E.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b$E.json')); print('$E envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bdef.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bdef.json')); print('default', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so
MAGENT_LIB=$L timeout -k 10 300 python scripts/stamps_few.py --envs 8 --sub 20 --launches 20 --snap > $O/stamps_few.txt 2>&1 || { tail -20 $O/stamps_few.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_few.txt
MAGENT_LIB=$L timeout -k 10 300 python scripts/stamps_battle.py --envs 8192 --steps 4 > $O/stamps8192.txt 2>&1 || { tail -20 $O/stamps8192.txt; exit 1; }
grep -v amdgpu.ids $O/stamps8192.txt
