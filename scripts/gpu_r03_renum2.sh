# Round 3: renumbering with the identity fast path -- parity, 256x256 A/B (interleaved), and the phase stamps
# of the few-env queue-kernel step (configs[3] shape: 8 envs of 64x64) from the MFX_STAMPS build.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/renum2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rollout_gpu.py \
    -k "large_env or bigq or small_e" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2 3; do
  for v in 0 1; do
    MFX_RENUMBER=$v timeout -k 10 300 python bench.py --map 256 --agents 4096 --no-cpu-baseline \
        > $O/ab_${v}_$r.json 2> $O/ab_${v}_$r.err || { tail -20 $O/ab_${v}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/ab_${v}_$r.json')); print('renumber=$v', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'kernel_ms %.3f' % d['roofline']['kernel_ms'], 'check', d['check']['ok'])"
  done
done
for e in 8 64; do
  MAGENT_LIB=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 200 \
      python scripts/stamps_big.py --map 64 --agents 256 --envs $e --steps 60 > $O/stamps_small_$e.txt 2>&1 || { tail -20 $O/stamps_small_$e.txt; exit 1; }
  cat $O/stamps_small_$e.txt
done
for s in 1 16; do
  timeout -k 10 300 python bench.py --total-envs 8 --substeps $s --no-cpu-baseline > $O/small8_s$s.json 2> $O/small8_s$s.err || { tail -20 $O/small8_s$s.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/small8_s$s.json')); print('8 envs substeps $s', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['roofline']['kernel'])"
done
