# Round 5: k_acnet instruction-cache counters (is the unrolled 512-wide layer fetch-bound?).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05ab}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_MFMA --output-format csv -d $GRAFT_REPO_ROOT/$O/ic -o a -- python3 $GRAFT_REPO_ROOT/scripts/bench_policy.py --net acnet --reps 3 > /dev/null 2> $GRAFT_REPO_ROOT/$O/err || { tail -20 $GRAFT_REPO_ROOT/$O/err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 - <<'PY'
import csv, glob, collections
for f in glob.glob('gpurun_out/r05ab/ic/**/*counter_collection.csv', recursive=True):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if 'k_acnet' in r['Kernel_Name']: agg[r['Counter_Name']] += float(r['Counter_Value'])
    for k, v in sorted(agg.items()): print(k, '%.4e' % v)
PY
