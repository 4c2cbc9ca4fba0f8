# Round 5: k_acnet phase costs (skip builds) + the 256x256 steps-per-launch threshold (2048 envs, S = 20..64).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05p}
mkdir -p $O
B=mean-field-multi-agent-reinforcement-learning_amd/build
for V in "" _skip1 _skip8 _skip9; do
MAGENT_LIB=$GRAFT_REPO_ROOT/$B/libmagent$V.so timeout -k 10 200 python scripts/bench_policy.py --net acnet > $O/acnet$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/acnet$V.json')); print('acnet$V ms %.3f tflops %.1f frac %.3f' % (d['ms_median'], d['tflops'], d['frac']))"
done
for S in 20 32 36 40 48 20; do
timeout -k 10 300 python bench.py --map 256 --substeps $S --steps 96 --warmup 16 --check-envs 2 --no-cpu-baseline > $O/s$S.json 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/s$S.json')); r=d['roofline']; print('S=$S %.4e frac %.4f ms/step %.4f kernel_ms %.3f check %s' % (d['value'], r['frac'], d['ms_per_step'], r.get('kernel_ms', -1), d.get('check', {}).get('ok')))"
done
