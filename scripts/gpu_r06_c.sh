# Round 6: packed view order with scalar descriptor prefetch; MFAC split lines; the forward alone; the bench line with
# the measured ceiling; Ising tests (guard, multi-pass, fallback) and the 2-rank Ising rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r06c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_policy_gpu.py -k "acnet or mfac" tests/test_ising_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for S in "" "--support"; do
timeout -k 10 200 python scripts/bench_policy.py --net acnet $S > $O/fwd$S.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/fwd$S.json')); print('acnet fwd [$S] ms %.3f frac %.4f' % (d['ms_median'], d['frac']))"
done
for V in "" "--split 2" "--split 2 --envs 16384" "--split 4 --envs 16384"; do
N=$(echo "$V" | tr -d ' -')
timeout -k 10 300 python bench.py --policy mfac --no-cpu-baseline $V > $O/mfac_$N.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/mfac_$N.json')); r=d['roofline']; print('mfac [$V]', '%.4e' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'fwd %.3f env %.3f' % (r['kernel_ms'], r['env_step_ms']), 'frac %.4f' % r['frac'], 'views', d['config']['view_inputs'])"
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('64x64', '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'measured_peak', r['measured_peak'], 'frac_measured', r['frac_measured'], r['measured_peak_detail']['per_shape_gbs'], 'check', d['check']['ok'])"
timeout -k 10 300 python scripts/bench_ising.py --mode reference --replicas 4096 --no-cpu --dump $O/ising1 > $O/ising1.json 2> $O/err || { tail -20 $O/err; exit 1; }
timeout -k 10 300 python scripts/bench_ising.py --mode reference --total-replicas 4096 --gpus 2 --backend gloo --no-cpu --dump $O/ising2 > $O/ising2.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 scripts/compare_ising_dumps.py $O/ising1 $O/ising2
python3 -c "import json; [print(k, (lambda d: (d['value'], d['ranks'], d['reduced'], d['check']))(json.load(open('$O/%s.json' % k)))) for k in ('ising1', 'ising2')]"
