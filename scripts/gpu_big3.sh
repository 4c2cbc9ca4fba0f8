set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py tests/test_battle_gpu.py > gpurun_out/big_tests.log 2>&1 || { tail -30 gpurun_out/big_tests.log; exit 1; }
timeout -k 10 300 python bench.py --map 256 --agents 4096 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/bench256.json 2> gpurun_out/bench256.err || exit 1
MAGENT_LIB=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 300 python scripts/stamps_big.py > gpurun_out/stamps_big.txt 2>&1 || exit 1
