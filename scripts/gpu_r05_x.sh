# Round 5: Ising stream mode with the passes double-buffered on two streams (MFX_ISING_OVERLAP A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05x}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ising_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for C in "16384 1" "16384 0" "4096 1" "256 1" "16384 1"; do
set -- $C; R=$1; V=$2
MFX_ISING_OVERLAP=$V timeout -k 10 300 python scripts/bench_ising.py --mode reference --replicas $R --no-cpu > $O/b${R}_$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b${R}_$V.json')); print('R=$R overlap=$V value %.4e call %.4f' % (d['value'], d['seconds_call']))"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o ising -- python3 $GRAFT_REPO_ROOT/scripts/bench_ising.py --mode reference --replicas 16384 --no-cpu > $GRAFT_REPO_ROOT/$O/bprof.json 2> $GRAFT_REPO_ROOT/$O/prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/ising_kernel_stats.csv')):
    if 'ising' in r['Name'] or 'mt_' in r['Name']: print('  ', r['Name'][:40], r['Calls'], '%.3f ms total' % (float(r['TotalDurationNs'])/1e6))
"
