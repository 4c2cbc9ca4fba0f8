# Round 5: the Ising scan at 256 words per chunk: tests, stats, kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05g}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ising_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
MFX_ISING_SCAN_STATS=1 timeout -k 10 200 python scripts/bench_ising.py --mode reference --no-cpu > $O/ising.json 2> $O/ising.err || { tail -20 $O/ising.err; exit 1; }
grep "ising scan" $O/ising.err | tail -1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o ising -- python3 $GRAFT_REPO_ROOT/scripts/bench_ising.py --mode reference --no-cpu > $GRAFT_REPO_ROOT/$O/bench.json 2> $GRAFT_REPO_ROOT/$O/prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 -c "
import csv, collections, json
d=json.load(open('$O/bench.json')); print('value %.4e call %.4f' % (d['value'], d['seconds_call']))
by=collections.defaultdict(list)
for r in csv.DictReader(open('$O/prof/ising_kernel_trace.csv')):
    by[r['Kernel_Name']].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6)
for k,v in by.items():
    if 'ising' in k or 'mt_' in k: print(k[:50], ['%.3f'%x for x in v])
"
