# Round 5: is the 256x256 line's 0.75 (last refresh) a regression from the wave-team work?  The build before it
# (commit 76e734f, build/libmagent_old.so) against the product build, alternating, same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05as}
mkdir -p $O
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
for R in 1 2 3; do
for V in _old ""; do
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 300 python bench.py --map 256 --agents 4096 --steps 20 --warmup 5 --no-cpu-baseline > $O/b256$V.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b256$V.json')); print('rep $R lib$V 256x256', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
done
done
