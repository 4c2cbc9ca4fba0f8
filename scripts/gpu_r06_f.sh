# Round 6: the envs as 2 engines on 2 streams in the rush bench (split) at 8192 / 16384 / 32768 / 131072 envs against one
# engine, same box, interleaved; the whole GPU suite on this tree (16-B row mover, wall-clock-bounded queue waits).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r06f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --durations=15 --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for r in 1 2; do
for E in 8192 16384 32768; do
for H in 1 2; do
timeout -k 10 200 python bench.py --total-envs $E --split $H --steps 256 --warmup 64 --no-cpu-baseline --check-envs 4 > $O/b_${E}_${H}_$r.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_${E}_${H}_$r.json')); r=d['roofline']; print('$E envs split $H', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'frac %.4f' % r['frac'], 'frac_measured %.4f' % r['frac_measured'], 'S', d['config']['steps_per_launch'], 'check', d['check']['ok'])"
done
done
for H in 1 2; do
timeout -k 10 400 python bench.py --split $H --steps 20 --warmup 5 --no-cpu-baseline --check-envs 4 > $O/b_def_${H}_$r.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_def_${H}_$r.json')); r=d['roofline']; print('131072 envs split $H', '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'frac_measured %.4f' % r['frac_measured'], 'check', d['check']['ok'])"
done
done
