# Round 3: the Q-network forward with its LDS operand reads software-pipelined (conv1, conv2, head): tests, bench, trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r03q3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_policy_gpu.py > $O/tests_policy.log 2>&1 || { tail -60 $O/tests_policy.log; exit 1; }
tail -1 $O/tests_policy.log
timeout -k 10 300 python bench.py --policy qnet --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_qnet.json 2> $O/bench_qnet.err || { tail -20 $O/bench_qnet.err; exit 1; }
cat $O/bench_qnet.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_qnet -o run --output-format csv -- python3 bench.py --policy qnet --steps 10 --warmup 2 > $O/prof_qnet.json 2> $O/prof_qnet.err || exit 1
head -6 $O/prof_qnet/run_kernel_stats.csv
