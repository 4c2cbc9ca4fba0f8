# Round 5: Ising stream mode defaults (64-GB passes, ring 24, two streams): tests, the default bench line, a trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05aa}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ising_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python scripts/bench_ising.py --mode reference > $O/bench_reference.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_reference.json')); print('reference R=%d value %.4e call %.4f check %s cpu %s' % (d['replicas'], d['value'], d['seconds_call'], d.get('check'), d.get('cpu_baseline', {}).get('value')))"
MFX_ISING_OVERLAP=0 timeout -k 10 300 python scripts/bench_ising.py --mode reference --no-cpu > $O/bench_ov0.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_ov0.json')); print('one stream value %.4e call %.4f' % (d['value'], d['seconds_call']))"
timeout -k 10 300 python scripts/bench_ising.py --mode philox --no-cpu > $O/bench_philox.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_philox.json')); print('philox value %.4e call %.4f' % (d['value'], d['seconds_call']))"
cd /tmp && MFX_ISING_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_ov0 -o ising -- python3 $GRAFT_REPO_ROOT/scripts/bench_ising.py --mode reference --no-cpu > /dev/null 2> $GRAFT_REPO_ROOT/$O/prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o ising -- python3 $GRAFT_REPO_ROOT/scripts/bench_ising.py --mode reference --no-cpu > /dev/null 2> $GRAFT_REPO_ROOT/$O/prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT && for P in prof_ov0 prof; do python3 -c "
import csv
print('$P')
for r in csv.DictReader(open('$O/$P/ising_kernel_stats.csv')):
    if 'ising' in r['Name'] or 'mt_' in r['Name']: print('  ', r['Name'][:40], r['Calls'], '%.3f ms total' % (float(r['TotalDurationNs'])/1e6))
"; done
