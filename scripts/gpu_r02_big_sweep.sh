# 256x256 (configs[4]) after the XCD-aware item lists: item-grid divisor sweep (MFX_ITEM_GRID_DIV),
# interleaved, two runs each.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02b
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for d in 3 2 4 6; do
    MFX_ITEM_GRID_DIV=$d timeout -k 10 200 python bench.py --map 256 --agents 4096 --steps 40 --warmup 5 --no-cpu-baseline > $O/d${d}_$r.json 2> $O/d${d}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/d${d}_$r.json')); print('div=$d', '%.4g'%d['value'], '%.3f'%d['roofline']['frac'])"
  done
done
