# tests + stamps on the current build, then A/B bench of libmagent_prev vs libmagent_cur on the same box
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests.log; exit 1; }
MAGENT_LIB=$B/libmagent_stamps.so timeout -k 10 300 python scripts/stamps_battle.py --envs 16384 > gpurun_out/stamps.txt 2>&1 || exit 1
bash scripts/gpu_variants.sh prev cur prev cur
