# Round 2 after the attack_big inlining fix: rollout parity, substeps sweep, profiles of the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rollout_gpu.py > $O/fixed_rollout_tests.log 2>&1 || { tail -30 $O/fixed_rollout_tests.log; exit 1; }
rm -f $O/sub_sweep2.jsonl
for i in 1 2; do for S in 1 2 4 8; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --substeps $S --steps 64 >> $O/sub_sweep2.jsonl 2>> $O/sub_sweep2.err || exit 1
done; done
bash scripts/gpu_r02_profiles.sh
