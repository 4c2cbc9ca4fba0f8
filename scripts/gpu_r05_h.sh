# Round 5: k_acnet with the view rows through LDS (A/B vs register staging); Ising kernel breakdown at 4096 / 16384.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_policy_gpu.py tests/test_ising_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for IMG in 0 1 0 1; do
MFX_ACNET_IMG=$IMG timeout -k 10 200 python scripts/bench_policy.py --net acnet > $O/acnet_img$IMG.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/acnet_img$IMG.json')); print('acnet img=$IMG ms %.3f tflops %.1f frac %.3f' % (d['ms_median'], d['tflops'], d['frac']))"
done
for R in 256 4096 16384; do
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof$R -o ising -- python3 $GRAFT_REPO_ROOT/scripts/bench_ising.py --mode reference --replicas $R --no-cpu > $GRAFT_REPO_ROOT/$O/bench$R.json 2> $GRAFT_REPO_ROOT/$O/prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 -c "
import csv, collections, json
d=json.load(open('$O/bench$R.json')); print('R=$R value %.4e call %.4f' % (d['value'], d['seconds_call']))
by=collections.defaultdict(float)
for r in csv.DictReader(open('$O/prof$R/ising_kernel_trace.csv')):
    by[r['Kernel_Name'][:40]] += (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6
for k,v in by.items():
    if 'ising' in k or 'mt_' in k: print('  ', k, '%.3f ms (all launches)' % v)
"
done
