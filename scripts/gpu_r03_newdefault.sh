# Round 3: the 64x64 bench default moves to 131072 envs x 8 steps per launch -- its oracle replay test, the
# default bench line (16-process CPU baseline), 131072 x 16 for comparison, kernel trace and PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/nd}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "bench_shape_matches_oracle or substeps_match" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('default', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'], 'cpu %.3e' % d['cpu_baseline']['value'], d['config']['envs_per_gpu'], d['config']['steps_per_launch'])"
for s in 16 8; do
timeout -k 10 300 python bench.py --substeps $s --steps 48 --warmup 16 --no-cpu-baseline > $O/s$s.json 2> $O/s$s.err || { tail -20 $O/s$s.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/s$s.json')); print('131072 x $s', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof64 -o run --output-format csv -- python3 bench.py --steps 48 --warmup 8 --no-cpu-baseline > $O/prof64.json 2> $O/prof64.err || exit 1
python3 scripts/timed_avg.py $O/prof64/run_kernel_trace.csv 6 > $O/timed_avg64.txt || exit 1
cat $O/timed_avg64.txt
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/f64 -o run --output-format csv -- python3 bench.py --steps 16 --warmup 8 --no-cpu-baseline --check-envs 0 > $O/f64.json 2> $O/f64.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/w64 -o run --output-format csv -- python3 bench.py --steps 16 --warmup 8 --no-cpu-baseline --check-envs 0 > $O/w64.json 2> $O/w64.err || exit 1
python3 scripts/summarize_prof.py $O/prof64 $O/f64 $O/w64 131072 $O/pmc_k_rollout.json 8 6 2 64 $O/prof64.json > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/pmc_k_rollout.json')); print({k: d[k] for k in ('hbm_bytes_per_agent_step', 'ratio', 'k_rollout_timed_avg_ns', 'bench_kernel_ms')})"
rm -f $O/f64/run_counter_collection.csv $O/w64/run_counter_collection.csv $O/prof64/run_kernel_trace.csv.bak
