#!/bin/bash
# Round 6: the workgroup team's attack internals in the few-env stepper (stamps builds, attack_team vs attack_big).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06n
mkdir -p $O
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
for v in stamps stamps_noteam; do
  MAGENT_LIB=$B/libmagent_$v.so timeout -k 10 300 python scripts/stamps_few.py --envs 8 --sub 20 --launches 20 > $O/$v.txt 2>&1 || { tail -20 $O/$v.txt; exit 1; }
  echo "== $v"; grep -E "agents|attack" $O/$v.txt
done
