#!/bin/bash
# Round 6 diagnostic: the eat-aware wave attack (variant build libmagent_foodpar${V:-}.so) against the reference build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06x
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_foodpar${V:-}.so
for c in "0 1 1 0 13" "0 1 0 1 14" "1 1 1 0 15"; do
  timeout -k 10 120 python -u scripts/diag_food.py $L $c >> gpurun_out/r06x/diag${V:-}.txt 2>&1 || exit 1
done
cat gpurun_out/r06x/diag${V:-}.txt | grep -v amdgpu.ids
