# 256x256 (configs[4]): the queue-driven large-env kernel (k_rollout_bigq) -- its parity tests first,
# then interleaved bench A/B against the two-stream pipeline (MFX_BIG_FUSED=0), item sizes
# (MFX_BIGQ_ROWS) and the stream's prefetch depth (libmagent_pf4.so, libmagent_pf3.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bigq
mkdir -p $O
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "large_env" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for v in q64 q128 q256 pf4 pf3 pipe; do
    lib=$L/libmagent.so; env="MFX_BIG_FUSED=1"
    case $v in
      q128) env="MFX_BIGQ_ROWS=128" ;;
      q256) env="MFX_BIGQ_ROWS=256" ;;
      pipe) env="MFX_BIG_FUSED=0" ;;
      pf4) lib=$L/libmagent_pf4.so ;;
      pf3) lib=$L/libmagent_pf3.so ;;
    esac
    env $env MAGENT_LIB=$lib timeout -k 10 200 python bench.py --map 256 --agents 4096 --steps 40 --warmup 5 --no-cpu-baseline > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$v', $r, '%.4g'%d['value'], '%.3f'%d['roofline']['frac'], '%.3f'%d['ms_per_step'])"
  done
done
