# Round 4: pipelined few-env form -- how much the idle item workers' polling costs the stepper: grid sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04h}
mkdir -p $O
export TMPDIR=/tmp
for E in 8 64; do for G in 0 256 128 64 32 16; do
  [ $E = 64 ] && [ $G -lt 128 ] && [ $G != 0 ] && continue
  MFX_BIGQ_GRID=$G timeout -k 10 200 python bench.py --total-envs $E --steps 200 --warmup 20 --no-cpu-baseline > $O/e${E}_g$G.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], 'grid', d['roofline']['grid'], '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_g$G.json
done; done
