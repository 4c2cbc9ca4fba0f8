# Round-2 refresh of the 256x256 line at 16 steps per launch: bench (16-core CPU baseline), kernel trace,
# FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r02k}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --map 256 --agents 4096 > $O/bench256.json 2> $O/bench256.err || { tail -20 $O/bench256.err; exit 1; }
cat $O/bench256.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 64 --warmup 16 --no-cpu-baseline > $O/prof256.json 2> $O/prof256.err || exit 1
python3 scripts/timed_avg.py $O/prof256/run_kernel_trace.csv 4 > $O/timed_avg256.txt || exit 1
cat $O/timed_avg256.txt
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 32 --warmup 16 --no-cpu-baseline > $O/f256.json 2> $O/f256.err || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 32 --warmup 16 --no-cpu-baseline > $O/w256.json 2> $O/w256.err || exit 1
python3 scripts/summarize_prof.py $O/prof256 $O/f256 $O/w256 1024 $O/pmc_big256.json 16 4 2 > /dev/null || exit 1
rm -f $O/f256/run_counter_collection.csv $O/w256/run_counter_collection.csv
