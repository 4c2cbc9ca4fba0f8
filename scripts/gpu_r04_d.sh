# Round 4: k_rollout with tiered queue start, one-ahead claims and restart-aware weights -- rollout tests, then the interleaved
# tiers (1), tiers without restart-aware weights (2), round-3 queue (0) A/B at 8192 / 131072 envs, and the 8192-env timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --durations=10 --timeout 300 --timeout-method thread -m gpu \
  tests/test_rollout_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for rep in 1 2; do for T in 1 2 0; do for E in 8192 131072; do
  MFX_QUEUE_TIERS=$T timeout -k 10 300 python bench.py --envs $E --steps 60 --warmup 10 --no-cpu-baseline --check-envs 2 > $O/e${E}_t$T.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], '%.4f' % d['roofline']['frac'], '%.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_t$T.json
done; done; done
L=mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so
MFX_QUEUE_TIERS=1 MAGENT_LIB=$L timeout -k 10 200 python scripts/timeline_rollout.py --envs 8192 --substeps 20 > $O/tl_8192_t1.txt 2>&1 || { tail -20 $O/tl_8192_t1.txt; exit 1; }
cat $O/tl_8192_t1.txt
