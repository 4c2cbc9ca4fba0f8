#!/bin/bash
# Round 6: food mode on the per-call step (serial attacks, the body kernel's wave moves / turns) -- rules tests, then same-box times vs the build before.
# attacks) -- rules tests against the reference build, the battle / rollout suites, then same-box step times against
# the build before the change (libmagent_prefood.so) and the reference engine.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06v
mkdir -p $O
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rules_gpu.py tests/test_battle_gpu.py tests/test_rollout_gpu.py \
  > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for cfg in "food 20 20,36" "turn_food 20 20,36" "turn 20 20,36" "double_attack 24 40,60"; do
    set -- $cfg
    for L in $B/libmagent.so $B/libmagent_prefood.so oracle/_ref/libmagent_ref.so; do
      timeout -k 10 120 python -u scripts/bench_generic.py --lib $L --config $1 --map $2 --counts $3 >> $O/times.jsonl 2>> $O/times.err || exit 1
      tail -1 $O/times.jsonl | cut -c1-170
    done
  done
done
