# Round 3: 20 steps per launch on every path -- the bench-shape oracle replays / pipeline test at 20, the default
# 64x64 and 256x256 lines (16-process CPU baseline), the driver-shaped line, kernel traces and PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/s20d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "bench_shape or small_e_matches" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('64 default', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'], 'cpu %.3e' % d['cpu_baseline']['value'])"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench_k20.err || { tail -20 $O/bench_k20.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_k20.json')); print('64 k20', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
timeout -k 10 400 python bench.py --map 256 --agents 4096 > $O/bench256.json 2> $O/bench256.err || { tail -20 $O/bench256.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench256.json')); print('256 default', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'], 'cpu %.3e' % d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof64 -o run --output-format csv -- python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline > $O/prof64.json 2> $O/prof64.err || exit 1
python3 scripts/timed_avg.py $O/prof64/run_kernel_trace.csv 3 > $O/timed_avg64.txt || exit 1
cat $O/timed_avg64.txt
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/f64 -o run --output-format csv -- python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --check-envs 0 > $O/f64.json 2> $O/f64.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/w64 -o run --output-format csv -- python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --check-envs 0 > $O/w64.json 2> $O/w64.err || exit 1
python3 scripts/summarize_prof.py $O/prof64 $O/f64 $O/w64 131072 $O/pmc_k_rollout.json 20 3 2 64 $O/prof64.json > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/pmc_k_rollout.json')); print({k: d[k] for k in ('hbm_bytes_per_agent_step', 'ratio', 'k_rollout_timed_avg_ns', 'bench_kernel_ms')})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 80 --warmup 20 --no-cpu-baseline > $O/prof256.json 2> $O/prof256.err || exit 1
python3 scripts/timed_avg.py $O/prof256/run_kernel_trace.csv 4 > $O/timed_avg256.txt || exit 1
cat $O/timed_avg256.txt
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/f256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 40 --warmup 20 --no-cpu-baseline --check-envs 0 > $O/f256.json 2> $O/f256.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/w256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 40 --warmup 20 --no-cpu-baseline --check-envs 0 > $O/w256.json 2> $O/w256.err || exit 1
python3 scripts/summarize_prof.py $O/prof256 $O/f256 $O/w256 2048 $O/pmc_big256.json 20 4 2 256 $O/prof256.json > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/pmc_big256.json')); print({k: d[k] for k in ('hbm_bytes_per_agent_step', 'ratio', 'k_rollout_timed_avg_ns', 'bench_kernel_ms')})"
rm -f $O/f64/run_counter_collection.csv $O/w64/run_counter_collection.csv $O/f256/run_counter_collection.csv $O/w256/run_counter_collection.csv
