set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py > gpurun_out/st_tests.log 2>&1 || { tail -30 gpurun_out/st_tests.log; exit 1; }
MAGENT_LIB=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 300 python scripts/stamps_big.py > gpurun_out/stamps_big.txt 2>&1 || exit 1
bash scripts/gpu_ab.sh head --map 256 --agents 4096 --steps 60 --warmup 5 > gpurun_out/ab_stage256.txt || exit 1
bash scripts/gpu_ab.sh head --steps 60 --warmup 5 > gpurun_out/ab_stage64.txt || exit 1
