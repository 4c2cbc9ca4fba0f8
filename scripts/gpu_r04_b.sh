# Round 4: the actor-critic forward (k_acnet), the sync-free Q-network act step, the pipelined replay mover and the
# tiered k_rollout queue start: GPU tests of the touched files, the learned-policy bench lines, replay variants,
# and the k_rollout batch-size sweep with tiers off / on (interleaved) plus launch timelines (stamp build).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --durations=15 --timeout 300 --timeout-method thread -m gpu \
  tests/test_policy_gpu.py tests/test_replay_gpu.py tests/test_rollout_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for T in 0 1; do for E in 8192 32768 131072; do
  MFX_QUEUE_TIERS=$T timeout -k 10 300 python bench.py --envs $E --steps 60 --warmup 10 --no-cpu-baseline --check-envs 2 > $O/e${E}_t$T.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], '%.4f' % d['roofline']['frac'], '%.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_t$T.json
done; done
L=mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so
for T in 0 1; do
MFX_QUEUE_TIERS=$T MAGENT_LIB=$L timeout -k 10 200 python scripts/timeline_rollout.py --envs 8192 --substeps 20 > $O/tl_8192_t$T.txt 2>&1 || { tail -20 $O/tl_8192_t$T.txt; exit 1; }
cat $O/tl_8192_t$T.txt
done
timeout -k 10 300 python bench.py --policy mfac --no-cpu-baseline > $O/bench_mfac.json 2> $O/err || { tail -20 $O/err; exit 1; }
cat $O/bench_mfac.json
timeout -k 10 300 python bench.py --policy qnet --no-cpu-baseline > $O/bench_qnet.json 2> $O/err || { tail -20 $O/err; exit 1; }
cat $O/bench_qnet.json
for V in "MFX_ROWS_PIPE=0" "MFX_ROWS_PIPE=1 MFX_ROWS_WG_PER_CU=4" "MFX_ROWS_PIPE=1 MFX_ROWS_WG_PER_CU=7" "MFX_ROWS_PIPE=1 MFX_ROWS_WG_PER_CU=14"; do
  env $V timeout -k 10 200 python scripts/bench_replay.py --cpu-seconds 1 > $O/replay.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4e' % d['value'], '%.1f' % d['roofline']['achieved'], '%.4f' % d['roofline']['frac'])" $O/replay.json "$V"
done
