#!/bin/bash
# Round 6: the reward DSL on the whole workgroup (dsl_rewards_team) -- rules tests against the reference build, then
# same-box per-call step times against the one-lane DFS (MFX_DSL_TEAM=0) and the reference engine.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06q
mkdir -p $O
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rules_gpu.py tests/test_battle_gpu.py \
  > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for cfg in "double_attack 24 40,60" "double_attack 40 20,64" "forest 32 60,50"; do
    set -- $cfg
    for L in $B/libmagent.so $B/libmagent_dslserial.so oracle/_ref/libmagent_ref.so; do
      timeout -k 10 120 python -u scripts/bench_generic.py --lib $L --config $1 --map $2 --counts $3 >> $O/times.jsonl 2>> $O/times.err || exit 1
      tail -1 $O/times.jsonl | cut -c1-220
    done
  done
done
