set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --map 256 --agents 4096 > gpurun_out/bench256.json 2> gpurun_out/bench256.err || { tail gpurun_out/bench256.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_big -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/prof_big.json 2> gpurun_out/prof_big.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_fetch.json 2> gpurun_out/pmc_fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_write.json 2> gpurun_out/pmc_write.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_big -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc_f_big.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_big -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc_w_big.err || exit 1
