# Round 3: the HIP Q-network forward (tests vs torch / float64, learned policy in the loop vs the oracle),
# the rollout tests after k_rollout's mode split, an A/B of k_rollout against the library before it, and the
# learned-policy bench line with its kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03q
mkdir -p $O
export TMPDIR=/tmp
L=mean-field-multi-agent-reinforcement-learning_amd/build
timeout -k 10 400 python -u -m pytest -x -v --durations=0 --timeout 280 --timeout-method thread -m gpu tests/test_policy_gpu.py > $O/tests_policy.log 2>&1 || { tail -60 $O/tests_policy.log; exit 1; }
grep -E "passed|failed" $O/tests_policy.log | tail -1
timeout -k 10 500 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_rollout_gpu.py > $O/tests_rollout.log 2>&1 || { tail -40 $O/tests_rollout.log; exit 1; }
tail -1 $O/tests_rollout.log
for r in 1 2 3; do for lib in libmagent_prev libmagent; do
MAGENT_LIB=$L/$lib.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 60 --warmup 8 > $O/ab_${lib}_$r.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/ab_${lib}_$r.json')); print('$lib', $r, '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], d['check']['ok'])"
done; done
timeout -k 10 300 python bench.py --policy qnet --steps 20 --warmup 3 > $O/bench_qnet.json 2> $O/bench_qnet.err || { tail -20 $O/bench_qnet.err; exit 1; }
cat $O/bench_qnet.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_qnet -o run --output-format csv -- python3 bench.py --policy qnet --steps 10 --warmup 2 > $O/prof_qnet.json 2> $O/prof_qnet.err || exit 1
head -8 $O/prof_qnet/run_kernel_stats.csv
