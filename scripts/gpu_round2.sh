# Full check after the large-env work: all GPU tests, smoke, 64x64 bench (+cpu baseline), 256x256 bench, profiles.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --map 256 --agents 4096 > gpurun_out/bench256.json 2> gpurun_out/bench256.err || { tail gpurun_out/bench256.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_big -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/prof_big.json 2> gpurun_out/prof_big.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_big -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc_f_big.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_big -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc_w_big.err || exit 1
