# Round 5: k_acnet phase costs (skip builds: 1 view GEMM, 8 h_emb recompute, 9 both).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05n}
mkdir -p $O
B=mean-field-multi-agent-reinforcement-learning_amd/build


for V in "" _skip1 _skip8 _skip9 ""; do
MAGENT_LIB=$GRAFT_REPO_ROOT/$B/libmagent$V.so timeout -k 10 200 python scripts/bench_policy.py --net acnet > $O/acnet$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/acnet$V.json')); print('acnet$V ms %.3f tflops %.1f frac %.3f' % (d['ms_median'], d['tflops'], d['frac']))"
done


