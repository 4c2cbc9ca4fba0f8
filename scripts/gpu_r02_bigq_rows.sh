# 256x256: k_rollout_bigq item size sweep (MFX_BIGQ_ROWS agents per observation item), interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bigq_rows
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for R in 256 384 512 1024; do
    MFX_BIGQ_ROWS=$R timeout -k 10 200 python bench.py --map 256 --agents 4096 --steps 40 --warmup 5 --no-cpu-baseline > $O/b_${R}_$r.json 2> $O/b_${R}_$r.err || { tail -20 $O/b_${R}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${R}_$r.json')); print('rows', $R, $r, '%.4g'%d['value'], '%.3f'%d['roofline']['frac'], '%.3f'%d['ms_per_step'])"
  done
done
