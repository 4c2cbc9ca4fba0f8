#!/bin/bash
# Round 6: 256x256 (configs[4], k_rollout_bigq, 2048 envs) as one engine vs two engines on two streams, two reps.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06w
mkdir -p $O
for r in 1 2; do
  for H in 1 2; do
    timeout -k 10 300 python bench.py --map 256 --agents 4096 --split $H --steps 20 --warmup 5 --no-cpu-baseline > $O/b256_s${H}_$r.json 2> $O/err || { tail -20 $O/err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b256_s${H}_$r.json')); r=d['roofline']; print('256 split $H', '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'frac_measured', r.get('frac_measured'), 'check', d['check']['ok'])"
  done
done
