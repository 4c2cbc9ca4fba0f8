# Round 5: Ising scan with the rolling LDS ring; scalar vs ballot walk at 256 / 4096 / 16384 replicas.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05i}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ising_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for R in 256 4096 16384; do
for S in 1 0; do
cd /tmp && MFX_ISING_SCAN_SALU=$S timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof${R}_$S -o ising -- python3 $GRAFT_REPO_ROOT/scripts/bench_ising.py --mode reference --replicas $R --no-cpu > $GRAFT_REPO_ROOT/$O/bench${R}_$S.json 2> $GRAFT_REPO_ROOT/$O/prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 -c "
import csv, collections, json
d=json.load(open('$O/bench${R}_$S.json')); print('R=$R salu=$S value %.4e call %.4f' % (d['value'], d['seconds_call']))
by=collections.defaultdict(float)
for r in csv.DictReader(open('$O/prof${R}_$S/ising_kernel_trace.csv')):
    by[r['Kernel_Name'][:40]] += (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6
for k,v in by.items():
    if 'ising' in k or 'mt_' in k: print('  ', k, '%.3f ms (all launches)' % v)
"
done
done
MFX_ISING_SCAN_STATS=1 timeout -k 10 120 python3 scripts/bench_ising.py --mode reference --replicas 256 --no-cpu 2>&1 >/dev/null | grep "ising scan" | head -3
