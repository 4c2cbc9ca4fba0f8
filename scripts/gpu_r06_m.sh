#!/bin/bash
# Round 6: attack_team (mask / chain form for <= 256 attackers on workgroup teams) -- parity of the rollout paths that
# take it, then same-box A/B against attack_big (MFX_ATTACK_TEAM=0 build): few-env stepper at 8 envs, 8192 envs,
# the headline; phase stamps of the few-env step.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06m
mkdir -p $O
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rollout_gpu.py tests/test_battle_gpu.py \
  > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1].split('/')[-1], '%.4e'%d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('check'))" $1; }
for r in 1 2; do
  for v in magent magent_noteam; do
    MAGENT_LIB=$B/lib$v.so timeout -k 10 180 python -u bench.py --envs 8 --steps 256 --warmup 64 --no-ceiling > $O/few_${v}_$r.json 2> $O/few_${v}_$r.err && show $O/few_${v}_$r.json || exit 1
    MAGENT_LIB=$B/lib$v.so timeout -k 10 180 python -u bench.py --envs 8192 --no-ceiling > $O/e8192_${v}_$r.json 2> $O/e8192_${v}_$r.err && show $O/e8192_${v}_$r.json || exit 1
  done
done
timeout -k 10 300 python -u bench.py --no-ceiling > $O/head.json 2> $O/head.err && show $O/head.json || exit 1
MAGENT_LIB=$B/libmagent_stamps.so timeout -k 10 300 python scripts/stamps_few.py --envs 8 --sub 20 --launches 20 --snap > $O/stamps_few.txt 2>&1 || { tail -20 $O/stamps_few.txt; exit 1; }
grep -E "agents|attack" $O/stamps_few.txt
