# Round 3: steps per launch on every bench path, at the driver's window (--steps 20 --warmup 5) and the default
# (--steps 60 --warmup 10): 64x64 k_rollout 8 vs 20, 256x256 k_rollout_bigq 16 vs 20, 8 envs (configs[3]) 16 vs 20.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sub20
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'ms/step %.4f' % d['ms_per_step'], 'check', d['check']['ok'])"
}
for r in 1 2; do
  for s in 8 20; do run 64_k60_s${s}_$r --substeps $s; done
  for s in 16 20; do run 256_k20_s${s}_$r --map 256 --agents 4096 --steps 20 --warmup 5 --substeps $s; done
  for s in 16 20; do run e8_k20_s${s}_$r --envs 8 --steps 20 --warmup 5 --substeps $s; done
done
for s in 16 20; do run 256_k60_s${s} --map 256 --agents 4096 --substeps $s; done
