# Round 5: numpy's Ising stream generated on the device -- the Ising GPU tests (every fixture through the device
# stream, device vs host stream, 2048 replicas vs the oracle), then the bench in every mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ising_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for M in reference host; do
timeout -k 10 300 python scripts/bench_ising.py --mode $M --no-cpu > $O/bench_$M.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_$M.json')); print('$M', '%.4e' % d['value'], 'R', d['replicas'], 'steps', d['steps_run'], 'call s %.4f' % d['seconds_call'], 'gen s %.2f' % d['host_stream_generation_s'], d.get('check'))"
done
for R in 4096 16384; do
timeout -k 10 300 python scripts/bench_ising.py --mode reference --replicas $R --no-cpu > $O/bench_reference_$R.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_reference_$R.json')); print('reference R=$R', '%.4e' % d['value'], 'call s %.4f' % d['seconds_call'], d.get('check'))"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o ising -- python3 $GRAFT_REPO_ROOT/scripts/bench_ising.py --mode reference --no-cpu > $GRAFT_REPO_ROOT/$O/bench_reference_prof.json 2> $GRAFT_REPO_ROOT/$O/prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head -3
