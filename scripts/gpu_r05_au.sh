# Round 5: the rollout row list (k_qnet_rows) over 64-env workgroups instead of one workgroup for the batch: the policy
# GPU tests on the variant, then product vs variant on the learned-policy loops (MF-Q, MFAC) with a kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05au}
mkdir -p $O
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
MAGENT_LIB=$B/libmagent_wave.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_policy_gpu.py > $O/tests_wave.log 2>&1 || { tail -30 $O/tests_wave.log; exit 1; }
tail -1 $O/tests_wave.log
for R in 1 2; do
for V in "" _wave; do
for P in mfac qnet; do
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 300 python bench.py --policy $P --no-cpu-baseline > $O/b_$P$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_$P$V.json')); print('rep $R lib$V $P', '%.4e' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'frac %.4f' % d['roofline']['frac'])"
done
done
done
MAGENT_LIB=$B/libmagent_wave.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --policy mfac --no-cpu-baseline --steps 10 --warmup 2 > $O/prof.json 2> $O/prof.err || exit 1
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof/run_kernel_stats.csv')))[:5]: print(r['Name'][:60], r['Calls'], '%.3f ms' % (float(r['AverageNs'])/1e6))
"
