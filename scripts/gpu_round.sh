# GPU session: parity tests, then a quick bench sweep. Each GPU step has its own time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/tests.log 2>&1 || { echo "tests failed"; exit 1; }
for E in 1024 4096; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --envs $E --no-cpu-baseline > gpurun_out/bench_E$E.json 2> gpurun_out/bench_E$E.err || exit 1
done
