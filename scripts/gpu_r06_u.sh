#!/bin/bash
# Round 6: the MF-Q loop as two engines on two streams (per-engine QNet handles) -- split 1 vs 2, two reps, same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06u
mkdir -p $O
for r in 1 2; do
  for H in 1 2; do
    timeout -k 10 300 python bench.py --policy qnet --split $H --no-cpu-baseline --no-ceiling > $O/qnet_s${H}_$r.json 2> $O/err || { tail -20 $O/err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/qnet_s${H}_$r.json')); r=d['roofline']; print('qnet split $H', '%.4e' % d['value'], 'ms/step %.2f' % d['ms_per_step'], 'fwd %.2f env %.2f' % (r['kernel_ms'], r['env_step_ms']), 'check', d['check']['ok'])"
  done
done
