# Round 3: steps per k_rollout launch at the driver's own window (--steps 20 --warmup 5): 8 (a 4-step remainder
# launch), 7 (balanced 7+7+6), 10 and 20 (whole launches), interleaved on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s20
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for s in 7 8 10 20; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --substeps $s --no-cpu-baseline > $O/s${s}_$r.json 2> $O/s${s}_$r.err || { tail -20 $O/s${s}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s${s}_$r.json')); print('steps 20 substeps $s', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
  done
done
