# iteration loop: parity tests -> stamps (diagnostic build) -> bench variants
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests.log; exit 1; }
MAGENT_LIB=$B/libmagent_stamps.so timeout -k 10 300 python scripts/stamps_battle.py --envs 16384 > gpurun_out/stamps.txt 2>&1 || exit 1
for V in ""; do
  for E in 16384; do
    MAGENT_LIB=$B/libmagent$V.so timeout -k 10 300 python bench.py --steps 50 --warmup 5 --envs $E --no-cpu-baseline > gpurun_out/bench$V.E$E.json 2> gpurun_out/bench.err || exit 1
  done
done
