# Round 4: k_acnet with h_emb recomputed from LDS (two workgroups per CU) vs held in registers; the k_rollout queue
# filed by predicted weight (episode restarts inside the next launch) with tiers; tests of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --durations=10 --timeout 300 --timeout-method thread -m gpu \
  tests/test_policy_gpu.py tests/test_rollout_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for H in 1 0 1 0; do
  MFX_ACNET_HE_LDS=$H timeout -k 10 300 python bench.py --policy mfac --no-cpu-baseline > $O/mfac_h$H.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], '%.4e' % d['value'], '%.2f TF/s' % r['achieved'], '%.4f' % r['frac'], '%.3f ms' % r['kernel_ms'])" $O/mfac_h$H.json "he_lds=$H"
done
for T in 1 0 1 0; do for E in 8192 131072; do
  MFX_QUEUE_TIERS=$T timeout -k 10 300 python bench.py --envs $E --steps 60 --warmup 10 --no-cpu-baseline --check-envs 2 > $O/e${E}_t$T.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], '%.4f' % d['roofline']['frac'], '%.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_t$T.json
done; done
L=mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so
MFX_QUEUE_TIERS=1 MAGENT_LIB=$L timeout -k 10 200 python scripts/timeline_rollout.py --envs 8192 --substeps 20 > $O/tl_8192_t1.txt 2>&1 || { tail -20 $O/tl_8192_t1.txt; exit 1; }
cat $O/tl_8192_t1.txt
for rep in 1 2; do
for V in "MFX_ROWS_PIPE=0" "MFX_ROWS_PIPE=1 MFX_ROWS_WG_PER_CU=4" "MFX_ROWS_PIPE=2 MFX_ROWS_WG_PER_CU=4" "MFX_ROWS_PIPE=2 MFX_ROWS_WG_PER_CU=8" "MFX_ROWS_PIPE=2 MFX_ROWS_NT=1 MFX_ROWS_WG_PER_CU=4" "MFX_ROWS_PIPE=3 MFX_ROWS_WG_PER_CU=6" "MFX_ROWS_PIPE=3 MFX_ROWS_NT=1 MFX_ROWS_WG_PER_CU=6"; do
  env $V timeout -k 10 200 python scripts/bench_replay.py --cpu-seconds 1 > $O/replay.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4e' % d['value'], '%.1f' % d['roofline']['achieved'], '%.4f' % d['roofline']['frac'])" $O/replay.json "$V"
done; done
