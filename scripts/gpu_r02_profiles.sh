# Round 2 profiles of the default bench (64x64, 24576 envs, 4 steps per k_rollout launch): full bench line
# with the 16-core CPU baseline, rocprofv3 kernel trace, FETCH_SIZE and WRITE_SIZE passes (one counter
# block per pass, MI355X_MICROARCH.md), summarised to gpurun_out/r02/pmc_k_rollout.json
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pf_prof -o run --output-format csv -- python3 bench.py --steps 60 --warmup 8 --no-cpu-baseline > $O/pf_prof.json 2> $O/pf_prof.err || exit 1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pf_fetch -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline > $O/pf_fetch.json 2> $O/pf_fetch.err || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pf_write -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline > $O/pf_write.json 2> $O/pf_write.err || exit 1
python3 scripts/summarize_prof.py $O/pf_prof $O/pf_fetch $O/pf_write 24576 $O/pmc_k_rollout.json 4 15 5 > /dev/null || exit 1
python3 scripts/timed_avg.py $O/pf_prof/run_kernel_trace.csv 15 > $O/timed_avg.txt || exit 1
rm -f $O/pf_fetch/run_counter_collection.csv.gz
cat $O/pmc_k_rollout.json | head -30
