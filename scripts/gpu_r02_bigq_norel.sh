# 256x256: k_rollout_bigq without the stepper's agent-scope release (libmagent_norel.so, A/B only: the
# consumers of an env's state run on its own XCD) -- its parity tests, then interleaved bench runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bigq_norel
mkdir -p $O
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
MAGENT_LIB=$L/libmagent_norel.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "large_env or bigq" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in base norel; do
    lib=$L/libmagent.so; [ $v != base ] && lib=$L/libmagent_$v.so
    MAGENT_LIB=$lib timeout -k 10 200 python bench.py --map 256 --agents 4096 --steps 48 --warmup 8 --no-cpu-baseline > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$v', $r, '%.4g'%d['value'], '%.3f'%d['roofline']['frac'], '%.3f'%d['ms_per_step'])"
  done
done
