# Round 3: the per-launch fixed cost -- 320 steps at 20 / 40 / 64 steps per launch (16 / 8 / 5 launches), 64x64
# (131072 envs) and 256x256 (2048 envs), interleaved, every line self-checked.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/slong
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 320 --warmup 10 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'ms/step %.4f' % d['ms_per_step'], 'launch ms %.3f' % d['roofline']['kernel_ms'], 'check', d['check']['ok'])"
}
for r in 1 2; do
  for s in 20 40 64; do run 64_s${s}_$r --substeps $s; done
  for s in 20 40 64; do run 256_s${s}_$r --map 256 --agents 4096 --substeps $s --check-envs 2; done
done
