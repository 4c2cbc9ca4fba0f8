# Round 3: the head's staged weights read with ds_read_b128 (build/libmagent_qhead.so) against the
# product library (vectorized Conv2, original Conv1): policy parity tests on it, kernel traces, two rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/qhead}
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build
MAGENT_LIB=$L/libmagent_qhead.so timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_policy_gpu.py > $O/tests_policy.log 2>&1 || { tail -60 $O/tests_policy.log; exit 1; }
tail -1 $O/tests_policy.log
for r in 1 2; do
  for v in product qhead; do
    if [ $v = product ]; then export MAGENT_LIB=$L/libmagent.so; else export MAGENT_LIB=$L/libmagent_$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${v}_$r -o run --output-format csv -- python3 bench.py --policy qnet --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_${v}_$r.json 2> $O/prof_${v}_$r.err || exit 1
    python3 -c "
import csv, json
for x in csv.DictReader(open('$O/prof_${v}_$r/run_kernel_stats.csv')):
    if 'qnet_conv' in x['Name'] or 'qnet_head' in x['Name']: print('$v r$r', x['Name'][5:20], '%.3f ms' % (float(x['AverageNs']) / 1e6))
d = json.load(open('$O/prof_${v}_$r.json')); print('$v r$r bench', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'])
"
    rm -f $O/prof_${v}_$r/run_kernel_trace.csv
  done
done
