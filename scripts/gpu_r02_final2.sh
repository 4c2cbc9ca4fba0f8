# Round-2 refresh after the queue-driven large-env kernel: GPU tests, smoke, the default bench line
# (16-core CPU baseline), the 256x256 line (k_rollout_bigq, 8 steps per launch) with its kernel trace
# and FETCH_SIZE / WRITE_SIZE passes, the 2-rank launcher rehearsal and configs[3].
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r02h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python bench.py --map 256 --agents 4096 > $O/bench256.json 2> $O/bench256.err || { tail -20 $O/bench256.err; exit 1; }
cat $O/bench256.json
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --envs 2048 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_2rank.json 2> $O/bench_2rank.err || { tail -20 $O/bench_2rank.err; exit 1; }
timeout -k 10 300 python bench.py --total-envs 64 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_64envs.json 2> $O/bench_64envs.err || { tail -20 $O/bench_64envs.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 64 --warmup 8 --no-cpu-baseline > $O/prof256.json 2> $O/prof256.err || exit 1
python3 scripts/timed_avg.py $O/prof256/run_kernel_trace.csv 8 > $O/timed_avg256.txt || exit 1
cat $O/timed_avg256.txt
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 32 --warmup 8 --no-cpu-baseline > $O/f256.json 2> $O/f256.err || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 32 --warmup 8 --no-cpu-baseline > $O/w256.json 2> $O/w256.err || exit 1
python3 scripts/summarize_prof.py $O/prof256 $O/f256 $O/w256 1024 $O/pmc_big256.json 8 8 4 > /dev/null || exit 1
rm -f $O/f256/run_counter_collection.csv $O/w256/run_counter_collection.csv
