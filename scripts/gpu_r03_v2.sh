# Round 3: rollout tests (paths, small-E, bench shapes), smoke, bench lines: default, configs[3] shape
# (8 and 64 envs on one GPU: the queue kernel), 256x256, and the 2-rank launcher rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03v2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --durations=0 --timeout 280 --timeout-method thread -m gpu tests/test_rollout_gpu.py > $O/tests_rollout.log 2>&1 || { tail -40 $O/tests_rollout.log; exit 1; }
grep -E "passed|failed" $O/tests_rollout.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
for E in 8 64; do
timeout -k 10 200 python bench.py --total-envs $E --steps 192 --warmup 16 --no-cpu-baseline > $O/bench_${E}envs.json 2> $O/err || { tail -20 $O/err; exit 1; }
cat $O/bench_${E}envs.json
done
timeout -k 10 400 python bench.py --map 256 --agents 4096 > $O/bench256.json 2> $O/bench256.err || { tail -20 $O/bench256.err; exit 1; }
cat $O/bench256.json
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --envs 2048 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_2rank.json 2> $O/bench_2rank.err || { tail -20 $O/bench_2rank.err; exit 1; }
cat $O/bench_2rank.json
