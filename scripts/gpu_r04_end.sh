# Round 4, end of the session: the whole GPU suite, smoke and the bench lines on the committed tree (the kernel traces
# and PMC passes of scripts/gpu_r04_final.sh stand: k_rollout and k_rollout_bigq<false> unchanged since).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04end}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --durations=15 --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('64x64', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'], 'cpu', '%.3e' % d['cpu_baseline']['value'])"
timeout -k 10 400 python bench.py --map 256 --agents 4096 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench256.json 2> $O/bench256.err || { tail -20 $O/bench256.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench256.json')); print('256x256', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
for E in 8 64 8192; do
timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/bench_${E}envs.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_${E}envs.json')); print('$E envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'frac %.4f' % d['roofline']['frac'], 'S', d['config']['steps_per_launch'], 'check', d['check']['ok'])"
done
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --total-envs 16 --steps 256 --warmup 64 --no-cpu-baseline > $O/bench_2rank_16envs.json 2> $O/e2.err || { tail -20 $O/e2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2rank_16envs.json')); print('2 ranks x 8 envs', '%.4e' % d['value'], d['config']['workload'], 'check', d['check']['ok'])"
timeout -k 10 200 python scripts/bench_dropin.py --map 40 --agents 128 --seconds 4 --calls > $O/dropin_40.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/dropin_40.json')); print('drop-in 40x40 vs ref', '%.3f' % d['hip_vs_ref'])"
