# Round 4: the hand-written actor-critic forward (k_acnet) and the sync-free Q-network act step: policy, replay
# and the new reference-pinned tests, the learned-policy bench lines, a kernel trace of the MFAC loop, and the
# k_rollout launch timeline (stamp build) at 8192 / 131072 envs.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04ac}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --durations=10 --timeout 300 --timeout-method thread -m gpu \
  tests/test_policy_gpu.py tests/test_replay_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 300 python bench.py --policy mfac --no-cpu-baseline > $O/bench_mfac.json 2> $O/err || { tail -20 $O/err; exit 1; }
cat $O/bench_mfac.json
timeout -k 10 300 python bench.py --policy qnet --no-cpu-baseline > $O/bench_qnet.json 2> $O/err || { tail -20 $O/err; exit 1; }
cat $O/bench_qnet.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mfac -o run --output-format csv -- python3 bench.py --policy mfac --no-cpu-baseline --steps 20 --warmup 3 > $O/prof_mfac.json 2> $O/prof_mfac.err || exit 1
python3 scripts/summarize_stats.py $O/prof_mfac/run_kernel_stats.csv 2>/dev/null | head -12 || head -12 $O/prof_mfac/run_kernel_stats.csv
L=mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so
for E in 8192 131072; do
MAGENT_LIB=$L timeout -k 10 200 python scripts/timeline_rollout.py --envs $E --substeps 20 > $O/tl_$E.txt 2>&1 || { tail -20 $O/tl_$E.txt; exit 1; }
cat $O/tl_$E.txt
done
for V in "MFX_ROWS_PIPE=0" "MFX_ROWS_PIPE=1 MFX_ROWS_WG_PER_CU=4" "MFX_ROWS_PIPE=1 MFX_ROWS_WG_PER_CU=7" "MFX_ROWS_PIPE=1 MFX_ROWS_WG_PER_CU=14"; do
  env $V timeout -k 10 200 python scripts/bench_replay.py --cpu-seconds 1 > $O/replay.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['achieved'], d['roofline']['frac'])" $O/replay.json "$V"
done
