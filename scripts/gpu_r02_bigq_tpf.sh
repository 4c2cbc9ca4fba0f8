# 256x256: k_rollout_bigq with 512-agent items -- ticket prefetch (libmagent_tpf.so) A/B, envs per GPU
# and steps per launch, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bigq_tpf
mkdir -p $O
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
for r in 1 2; do
  for v in base tpf e2048 e1536 s8; do
    lib=$L/libmagent.so; args=""
    case $v in
      tpf) lib=$L/libmagent_tpf.so ;;
      e2048) args="--envs 2048" ;;
      e1536) args="--envs 1536" ;;
      s8) args="--substeps 8" ;;
    esac
    MAGENT_LIB=$lib timeout -k 10 200 python bench.py --map 256 --agents 4096 --steps 40 --warmup 5 --no-cpu-baseline $args > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$v', $r, '%.4g'%d['value'], '%.3f'%d['roofline']['frac'], '%.3f'%d['ms_per_step'])"
  done
done
