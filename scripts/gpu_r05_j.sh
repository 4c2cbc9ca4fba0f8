# Round 5: Ising scan ring size A/B (16 / 32 / 64 blocks) at 256 / 4096 / 16384 replicas; k_acnet SQ counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05j}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ising_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for R in 16384 4096 256; do
for RB in 32 16 64; do
cd /tmp && MFX_ISING_SCAN_RING=$RB timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof${R}_$RB -o ising -- python3 $GRAFT_REPO_ROOT/scripts/bench_ising.py --mode reference --replicas $R --no-cpu > $GRAFT_REPO_ROOT/$O/bench${R}_$RB.json 2> $GRAFT_REPO_ROOT/$O/prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 -c "
import csv, collections, json
d=json.load(open('$O/bench${R}_$RB.json')); print('R=$R ring=$RB value %.4e call %.4f' % (d['value'], d['seconds_call']))
by=collections.defaultdict(float)
for r in csv.DictReader(open('$O/prof${R}_$RB/ising_kernel_trace.csv')):
    by[r['Kernel_Name'][:40]] += (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6
for k,v in by.items():
    if 'ising' in k or 'mt_' in k: print('  ', k, '%.3f ms (all launches)' % v)
"
done
done
MFX_ISING_SCAN_STATS=1 timeout -k 10 120 python3 scripts/bench_ising.py --mode reference --replicas 4096 --no-cpu 2>&1 >/dev/null | grep "ising scan" | head -3
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc1 -o acnet -- python3 $GRAFT_REPO_ROOT/scripts/bench_policy.py --net acnet --reps 3 > $GRAFT_REPO_ROOT/$O/pmc1.json 2>$GRAFT_REPO_ROOT/$O/pmc.err || { tail -20 $GRAFT_REPO_ROOT/$O/pmc.err; exit 1; }
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc2 -o acnet -- python3 $GRAFT_REPO_ROOT/scripts/bench_policy.py --net acnet --reps 3 > $GRAFT_REPO_ROOT/$O/pmc2.json 2>$GRAFT_REPO_ROOT/$O/pmc.err || { tail -20 $GRAFT_REPO_ROOT/$O/pmc.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 - <<'PY'
import csv, glob, collections
for d in ('pmc1', 'pmc2'):
    for f in glob.glob('gpurun_out/r05j/%s/**/*counter_collection.csv' % d, recursive=True):
        agg = collections.defaultdict(float); n = collections.Counter()
        for r in csv.DictReader(open(f)):
            if 'k_acnet' not in r['Kernel_Name']: continue
            agg[r['Counter_Name']] += float(r['Counter_Value'])
        for k, v in sorted(agg.items()): print(d, k, '%.4e' % v)
PY
