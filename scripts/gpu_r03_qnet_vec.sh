# Round 3: the vectorized Conv2 (permuted k order, transposed weights, ds_read_b128, reads of the next block
# interleaved in two parts) + the pipelined head, as build/libmagent_qvec.so: the policy parity tests on it, then
# kernel traces interleaved with the previous form (qold), two rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/qvec}
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build
MAGENT_LIB=$L/libmagent_qvec.so timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_policy_gpu.py > $O/tests_policy.log 2>&1 || { tail -60 $O/tests_policy.log; exit 1; }
tail -2 $O/tests_policy.log
for r in 1 2; do
  for v in qold qvec qc1 qc2 new; do
    [ $r = 2 ] && [ $v != qold ] && [ $v != qvec ] && continue
    if [ $v = new ]; then export MAGENT_LIB=$L/libmagent.so; else export MAGENT_LIB=$L/libmagent_$v.so; fi
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
