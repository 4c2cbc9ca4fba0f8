set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py tests/test_battle_gpu.py tests/test_rules_gpu.py > gpurun_out/wj_tests.log 2>&1 || { tail -30 gpurun_out/wj_tests.log; exit 1; }
MAGENT_LIB=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 300 python scripts/stamps_battle.py --envs 16384 > gpurun_out/stamps64.txt 2>&1 || exit 1
bash scripts/gpu_ab.sh head --steps 60 --warmup 5 > gpurun_out/ab_wj.txt || exit 1
