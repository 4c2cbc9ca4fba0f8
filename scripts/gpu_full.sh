# Full GPU session: tests -> smoke -> bench (+cpu baseline) -> rocprofv3 trace -> PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_fetch.json 2> gpurun_out/pmc_fetch.err || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_write.json 2> gpurun_out/pmc_write.err || exit 1
