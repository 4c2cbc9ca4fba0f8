set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused -o run --output-format csv -- python3 scripts/prof_battle.py --mode fused --envs 4096 --steps 20 > gpurun_out/prof_fused.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_percall -o run --output-format csv -- python3 scripts/prof_battle.py --mode percall --envs 4096 --steps 20 > gpurun_out/prof_percall.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --envs 4096 --no-cpu-baseline > gpurun_out/bench_E4096.json 2> gpurun_out/bench.err || exit 1
