# Round 5: k_qnet_conv2 (two waves per agent, two per SIMD) vs k_qnet_conv (MFX_QNET_CONV=1): parity, forward, loop.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05ai}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_policy_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for C in 0 1 0 1; do
MFX_QNET_CONV=$C timeout -k 10 200 python scripts/bench_policy.py --net qnet > $O/q$C.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/q$C.json')); print('qnet conv_old=$C ms %.3f tflops %.1f frac %.3f' % (d['ms_median'], d['tflops'], d['frac']))"
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o q -- python3 $GRAFT_REPO_ROOT/scripts/bench_policy.py --net qnet --reps 5 > /dev/null 2> $GRAFT_REPO_ROOT/$O/prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/q_kernel_stats.csv')):
    if 'qnet' in r['Name']: print('  ', r['Name'][:40], r['Calls'], '%.3f ms avg' % (float(r['AverageNs'])/1e6))
"
timeout -k 10 400 python bench.py --policy qnet --no-cpu-baseline > $O/bench_qnet.json 2> $O/bench_qnet.err || { tail -20 $O/bench_qnet.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_qnet.json')); r=d['roofline']; print('qnet loop value %.4e ms/step %.3f' % (d['value'], d['ms_per_step']), r['frac'], r['kernel_ms'])"
