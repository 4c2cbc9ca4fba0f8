# Round 4: observation item size of the pipelined few-env form (MFX_BIGQ_ROWS, default 16 agents per item).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04ae}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do for R in 8 16 32; do for E in 8 64; do
  MFX_BIGQ_ROWS=$R timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/e${E}_r$R.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_r$R.json
done; done; done
