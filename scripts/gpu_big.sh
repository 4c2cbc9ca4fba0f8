# Large-env path: parity (per-call k_step_big via the 256x256 fixture, k_rollout_big lockstep) then bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_battle_gpu.py tests/test_rollout_gpu.py > gpurun_out/big_tests.log 2>&1 || { tail -40 gpurun_out/big_tests.log; exit 1; }
timeout -k 10 300 python bench.py --map 256 --agents 4096 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench256.json 2> gpurun_out/bench256.err || { tail gpurun_out/bench256.err; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench64.json 2> gpurun_out/bench64.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_big -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 20 --warmup 3 --no-cpu-baseline --max-steps 100 > gpurun_out/prof_big.json 2> gpurun_out/prof_big.err || exit 1
