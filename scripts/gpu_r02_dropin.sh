# Round 2: the fast drop-in step -- parity (fixtures, random scenarios, odd call orders), then timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02
export TMPDIR=/tmp
O=gpurun_out/r02
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_battle_gpu.py -k "odd_call or replays_reference_fixture or random_scenarios" > $O/dropin_tests.log 2>&1 || { tail -40 $O/dropin_tests.log; exit 1; }
for m in "40 128" "64 256"; do
  set -- $m
  MFX_DROPIN_FAST=1 timeout -k 10 120 python scripts/bench_dropin.py --map $1 --agents $2 --calls >> $O/dropin_bench.jsonl 2>> $O/dropin_bench.err || exit 1
  MFX_DROPIN_FAST=0 timeout -k 10 120 python scripts/bench_dropin.py --map $1 --agents $2 --calls >> $O/dropin_bench.jsonl 2>> $O/dropin_bench.err || exit 1
done
