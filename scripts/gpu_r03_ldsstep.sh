# Round 3: the few-env path stages each env in LDS for its step (RolloutArgs::lds_step).  Parity of every
# queue-kernel test, then configs[3]-shape A/B (MFX_LDS_STEP=0 / 1 interleaved) at 8 and 64 envs, and the
# 256x256 default once (its layout lost the unused claim table only where acap <= 4096 ... unchanged here).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/ldsstep}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rollout_gpu.py \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for e in 8 64; do
    for v in 0 1; do
      MFX_LDS_STEP=$v timeout -k 10 300 python bench.py --total-envs $e --no-cpu-baseline > $O/ab_${e}_${v}_$r.json 2> $O/ab_${e}_${v}_$r.err || { tail -20 $O/ab_${e}_${v}_$r.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/ab_${e}_${v}_$r.json')); print('envs $e lds_step=$v', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['roofline']['kernel'], 'check', d['check']['ok'])"
    done
  done
done
timeout -k 10 300 python bench.py --map 256 --agents 4096 --no-cpu-baseline > $O/b256.json 2> $O/b256.err || { tail -20 $O/b256.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b256.json')); print('256x256', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
