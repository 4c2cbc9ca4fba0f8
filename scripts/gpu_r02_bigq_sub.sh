# 256x256: k_rollout_bigq steps per launch and envs per GPU, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bigq_sub
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in s8 s16 e768s8 e512s8 s8r384; do
    env="MFX_BIG_FUSED=1"; args=""
    case $v in
      s8) args="--substeps 8" ;;
      s16) args="--substeps 16 --steps 48" ;;
      e768s8) args="--envs 768 --substeps 8" ;;
      e512s8) args="--envs 512 --substeps 8" ;;
      s8r384) args="--substeps 8"; env="MFX_BIGQ_ROWS=384" ;;
    esac
    env $env timeout -k 10 200 python bench.py --map 256 --agents 4096 --steps 40 --warmup 8 --no-cpu-baseline $args > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$v', $r, '%.4g'%d['value'], '%.3f'%d['roofline']['frac'], '%.3f'%d['ms_per_step'])"
  done
done
