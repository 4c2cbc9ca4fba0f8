# Round 5: Ising scan (per-lane-mask walk, 32-block ring); persistent k_acnet A/B; MFAC loop.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05k}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ising_gpu.py tests/test_policy_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for R in 16384 4096 256; do
for RB in 32 64; do
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
for P in 1 0 1; do
MFX_ACNET_PERSIST=$P timeout -k 10 200 python scripts/bench_policy.py --net acnet > $O/acnet_p$P.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/acnet_p$P.json')); print('acnet persist=$P ms %.3f tflops %.1f frac %.3f' % (d['ms_median'], d['tflops'], d['frac']))"
done
timeout -k 10 400 python bench.py --policy mfac --no-cpu-baseline > $O/bench_mfac.json 2> $O/bench_mfac.err || { tail -20 $O/bench_mfac.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_mfac.json')); print('mfac value %.4e ms/step %.3f' % (d['value'], d['ms_per_step']))"
