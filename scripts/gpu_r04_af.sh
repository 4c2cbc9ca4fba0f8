# Round 4: steps per launch at 256x256 (2048 envs, k_rollout_bigq): is the engine's 20 still the best?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04af}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do for S in 10 16 20 24 32; do
  timeout -k 10 300 python bench.py --map 256 --agents 4096 --substeps $S --steps 96 --warmup 16 --no-cpu-baseline --check-envs 2 > $O/s$S.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], d['check']['ok'])" $O/s$S.json
done; done
