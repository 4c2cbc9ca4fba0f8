# Refresh profiles/pmc_k_rollout.json for the current tree (default bench config):
# kernel trace, then separate FETCH_SIZE / WRITE_SIZE passes, summarised by summarize_prof.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pf_prof -o run --output-format csv -- python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/pf_prof.json 2> gpurun_out/pf_prof.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pf_fetch -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/pf_fetch.json 2> gpurun_out/pf_fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pf_write -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/pf_write.json 2> gpurun_out/pf_write.err || exit 1
python3 scripts/summarize_prof.py gpurun_out/pf_prof gpurun_out/pf_fetch gpurun_out/pf_write 24576 gpurun_out/pmc_final.json > /dev/null || exit 1
rm -f gpurun_out/pf_*/run_kernel_trace.csv gpurun_out/pf_*/run_counter_collection.csv
cat gpurun_out/pmc_final.json
