# Round 5: bench.py with no flags (the driver's default invocation) on the final tree, timed by the shell.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05ax}
mkdir -p $O
S=$(date +%s)
timeout -k 10 600 python bench.py > $O/bench_noflags.json 2> $O/bench_noflags.err || { tail -20 $O/bench_noflags.err; exit 1; }
echo "wall $(( $(date +%s) - S )) s"
python3 -c "import json; d=json.load(open('$O/bench_noflags.json')); print(d['metric'], '%.4e' % d['value'], d['steps'], d['warmup'], 'frac %.4f' % d['roofline']['frac'], 'cpu %.3e' % d['cpu_baseline']['value'], 'check', d['check']['ok'])"
