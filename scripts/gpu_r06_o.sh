#!/bin/bash
# Round 6: kill_supply configs on the parallel forms (the per-call step's supply-aware wave attack) -- the rules
# tests against the reference build, the battle / rollout suites, then same-box step times against the serial
# build (MFX_SUPPLY_PAR=0) and the reference engine.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06o
mkdir -p $O
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rules_gpu.py tests/test_battle_gpu.py tests/test_rollout_gpu.py \
  > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for cfg in "double_attack 24 40,60" "forest 32 60,50" "double_attack 40 20,64"; do
    set -- $cfg
    for L in $B/libmagent.so $B/libmagent_supserial.so oracle/_ref/libmagent_ref.so; do
      timeout -k 10 120 python -u scripts/bench_generic.py --lib $L --config $1 --map $2 --counts $3 >> $O/times.jsonl 2>> $O/times.err || exit 1
      tail -1 $O/times.jsonl
    done
  done
done
