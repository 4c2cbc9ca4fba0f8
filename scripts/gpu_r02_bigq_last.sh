# 256x256, k_rollout_bigq without the per-step L2 write-back: steps per launch, item size, envs per GPU,
# interleaved, 2 runs each.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bigq_last
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in base s16 r256 e1536; do
    env="MFX_BIG_FUSED=1"; args=""
    case $v in
      s16) args="--substeps 16" ;;
      r256) env="MFX_BIGQ_ROWS=256" ;;
      e1536) args="--envs 1536" ;;
    esac
    env $env timeout -k 10 200 python bench.py --map 256 --agents 4096 --steps 48 --warmup 8 --no-cpu-baseline $args > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$v', $r, '%.4g'%d['value'], '%.3f'%d['roofline']['frac'], '%.3f'%d['ms_per_step'])"
  done
done
