# 256x256: k_rollout_bigq stream prefetch depth with 512-agent items (default 6; libmagent_pf8.so,
# libmagent_pf4.so), interleaved, 2 runs each.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bigq_pf
mkdir -p $O
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
for r in 1 2; do
  for v in base pf8 pf4; do
    lib=$L/libmagent.so; [ $v != base ] && lib=$L/libmagent_$v.so
    MAGENT_LIB=$lib timeout -k 10 200 python bench.py --map 256 --agents 4096 --steps 48 --warmup 8 --no-cpu-baseline > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$v', $r, '%.4g'%d['value'], '%.3f'%d['roofline']['frac'], '%.3f'%d['ms_per_step'])"
  done
done
