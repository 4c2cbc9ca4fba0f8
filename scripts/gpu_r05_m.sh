# Round 5: k_acnet phase costs from skip builds (A/B only: libmagent_skipN.so skips view 1 / dense 2 / policy 4).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05m}
mkdir -p $O
B=mean-field-multi-agent-reinforcement-learning_amd/build
for V in "" _skip1 _skip2 _skip4 ""; do
MAGENT_LIB=$GRAFT_REPO_ROOT/$B/libmagent$V.so timeout -k 10 200 python scripts/bench_policy.py --net acnet > $O/acnet$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/acnet$V.json')); print('acnet$V ms %.3f tflops %.1f frac %.3f' % (d['ms_median'], d['tflops'], d['frac']))"
done
