# Round 3: 256x256 steps per k_rollout_bigq launch after the slot renumbering -- 16 (default) vs 32 vs 64,
# interleaved on one box, every line self-checked on the oracle.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/sub256}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for s in 16 32 64; do
    timeout -k 10 300 python bench.py --map 256 --agents 4096 --substeps $s --steps 128 --warmup 16 --no-cpu-baseline > $O/s${s}_$r.json 2> $O/s${s}_$r.err || { tail -20 $O/s${s}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s${s}_$r.json')); print('substeps $s', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
  done
done
