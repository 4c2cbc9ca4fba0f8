# Round 3: the few-env queue kernel's one-wave agent phase (k_rollout_bigq<true>, lds_step 1) -- parity of the
# rollout tests, then an interleaved A/B at 8 and 64 envs: MFX_LDS_STEP=0 (HBM step), 2 (LDS step, no wave
# phase), 1 (LDS step + one-wave phase for <= 64 agents); every line self-checked on the oracle.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/wave}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rollout_gpu.py \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for e in 8 64 512; do
    for v in 0 2 1; do
      MFX_LDS_STEP=$v timeout -k 10 300 python bench.py --total-envs $e --no-cpu-baseline > $O/ab_${e}_${v}_$r.json 2> $O/ab_${e}_${v}_$r.err || { tail -20 $O/ab_${e}_${v}_$r.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/ab_${e}_${v}_$r.json')); print('envs $e lds_step=$v', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['roofline']['kernel'], 'grid', d['roofline'].get('grid'), 'check', d['check']['ok'])"
    done
  done
done
