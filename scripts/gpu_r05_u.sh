# Round 5: 8192 envs at 64x64 -- k_rollout at 1 / 2 / 4 / 8 steps per launch against the queue kernel (MFX_SMALL_E=8192:
# observation items shared by every workgroup of an XCD, the step by the env's last finisher, env staged in LDS).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05u}
mkdir -p $O
run() {
  timeout -k 10 300 python bench.py --envs 8192 --no-cpu-baseline "$@" > $O/x.json 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/x.json')); r=d['roofline']; print(sys.argv[1], '%.4e frac %.4f ms/step %.4f kernel %s spl %s check %s' % (d['value'], r['frac'], d['ms_per_step'], r.get('kernel'), d['config'].get('steps_per_launch'), d.get('check', {}).get('ok')))" "$*"
}
run --substeps 2
run --substeps 4
run --substeps 1
MFX_SMALL_E=8192 run --substeps 20
MFX_SMALL_E=8192 run --substeps 8
MFX_SMALL_E=8192 MFX_BIGQ_ROWS=64 run --substeps 20
run --substeps 2
