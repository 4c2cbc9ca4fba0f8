# Round 3: the 256x256 bench default moves to 2048 envs -- the bench-shape oracle replay and pipeline tests at
# that shape, the default 256x256 line (16-process CPU baseline), kernel trace and PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/nd256}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "bigq_bench_shape" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 400 python bench.py --map 256 --agents 4096 > $O/bench256.json 2> $O/bench256.err || { tail -20 $O/bench256.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench256.json')); print('256 default', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'], 'cpu %.3e' % d['cpu_baseline']['value'], d['config']['envs_per_gpu'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 64 --warmup 16 --no-cpu-baseline > $O/prof256.json 2> $O/prof256.err || exit 1
python3 scripts/timed_avg.py $O/prof256/run_kernel_trace.csv 4 > $O/timed_avg256.txt || exit 1
cat $O/timed_avg256.txt
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/f256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 32 --warmup 16 --no-cpu-baseline --check-envs 0 > $O/f256.json 2> $O/f256.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/w256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 32 --warmup 16 --no-cpu-baseline --check-envs 0 > $O/w256.json 2> $O/w256.err || exit 1
python3 scripts/summarize_prof.py $O/prof256 $O/f256 $O/w256 2048 $O/pmc_big256.json 16 4 2 256 $O/prof256.json > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/pmc_big256.json')); print({k: d[k] for k in ('hbm_bytes_per_agent_step', 'ratio', 'k_rollout_timed_avg_ns', 'bench_kernel_ms')})"
rm -f $O/f256/run_counter_collection.csv $O/w256/run_counter_collection.csv
