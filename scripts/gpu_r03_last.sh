# Round 3: last check of the committed tree -- the whole GPU suite, smoke, the default bench line and the
# learned-policy line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r03last}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --durations=10 --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('64x64', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'traffic', d['roofline']['traffic'], 'check', d['check']['ok'], 'cpu', '%.3e' % d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --policy qnet --no-cpu-baseline > $O/bench_qnet.json 2> $O/bench_qnet.err || { tail -20 $O/bench_qnet.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_qnet.json')); print('qnet', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'])"
