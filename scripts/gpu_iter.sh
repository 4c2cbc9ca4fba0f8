# iteration loop: parity tests -> stamps (diagnostic build) -> bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests.log; exit 1; }
MAGENT_LIB=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 300 python scripts/stamps_battle.py --envs 4096 > gpurun_out/stamps.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --envs 4096 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
