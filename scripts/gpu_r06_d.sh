# Round 6: the whole GPU suite on the round's first commit, the default bench line (measured ceiling), the MFAC default
# line, the 2-rank Ising rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r06d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --durations=15 --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('64x64', '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'measured_peak %.0f' % r['measured_peak'], 'frac_measured %.4f' % r['frac_measured'], {k: round(v) for k, v in r['measured_peak_detail']['per_shape_gbs'].items()}, 'check', d['check']['ok'], 'traffic', r['traffic'])"
timeout -k 10 300 python bench.py --policy mfac --no-cpu-baseline > $O/mfac.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/mfac.json')); r=d['roofline']; print('mfac', '%.4e' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'fwd %.3f env %.3f' % (r['kernel_ms'], r['env_step_ms']), 'frac %.4f' % r['frac'], d['config']['engines'])"
timeout -k 10 300 python scripts/bench_ising.py --mode reference --total-replicas 4096 --gpus 2 --backend gloo --no-cpu --dump $O/ising2 > $O/ising2.json 2> $O/err || { tail -20 $O/err; exit 1; }
timeout -k 10 300 python scripts/bench_ising.py --mode reference --replicas 4096 --no-cpu --dump $O/ising1 > $O/ising1.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 scripts/compare_ising_dumps.py $O/ising1 $O/ising2 | tee $O/ising_compare.json
python3 -c "import json; [print(k, (lambda d: (d['value'], d['ranks'], d['parallelism'], d['reduced'], d['check']['mismatches']))(json.load(open('$O/%s.json' % k)))) for k in ('ising1', 'ising2')]"
