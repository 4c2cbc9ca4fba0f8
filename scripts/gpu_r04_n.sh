# Round 4: the chunked mid-size attack (attack_chunked: workgroup shuffle, 64-attack chunks on wave 0) -- the whole
# GPU suite, the stepper's stamps, then A/B against the build without it (MFX_ATTACK_CHUNKED_MAX=0) at configs[3]
# shapes, 8192 envs and the bench default.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04n}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
MAGENT_LIB=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 200 \
    python scripts/stamps_few.py --envs 8 > $O/stamps_8.txt 2>&1 || { tail -20 $O/stamps_8.txt; exit 1; }
grep -E "pipelined|agents:" $O/stamps_8.txt
L=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build
for rep in 1 2; do for V in product nochunk; do
  if [ $V = product ]; then LIB=$L/libmagent.so; else LIB=$L/libmagent_nochunk.so; fi
  for E in 8 64 8192; do
    MAGENT_LIB=$LIB timeout -k 10 200 python bench.py --total-envs $E --steps 100 --warmup 20 --no-cpu-baseline > $O/e${E}_$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_$V.json
  done
done; done
for V in product nochunk; do
  if [ $V = product ]; then LIB=$L/libmagent.so; else LIB=$L/libmagent_nochunk.so; fi
  MAGENT_LIB=$LIB timeout -k 10 300 python bench.py --no-cpu-baseline > $O/def_$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/def_$V.json
done
