# Round 6: the multi-rank flow on the reworked bench (engines, fork / join, per-engine checks): 2-rank gloo rehearsals
# (default envs per rank at 2048, the split at 8192, configs[3]'s 16 envs); smoke(); bench.py with no flags.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r06h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --envs 2048 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_2rank.json 2> $O/bench_2rank.err || { tail -20 $O/bench_2rank.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2rank.json')); print('2 ranks x 2048', '%.4e' % d['value'], d['n_gpus'], d['ranks'], d['config']['parallelism'], d['config']['engines'], d['check']['ok'], d['check']['envs'], d['episodes']['note'])"
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --envs 8192 --steps 64 --warmup 8 --no-cpu-baseline > $O/bench_2rank_split.json 2> $O/bench_2rank_split.err || { tail -20 $O/bench_2rank_split.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2rank_split.json')); print('2 ranks x 8192 (2 engines each)', '%.4e' % d['value'], d['config']['engines'], d['check']['ok'], d['check']['envs'], d['episodes'])"
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --total-envs 16 --steps 256 --warmup 64 --no-cpu-baseline > $O/bench_2rank_16envs.json 2> $O/bench_2rank_16envs.err || { tail -20 $O/bench_2rank_16envs.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2rank_16envs.json')); print('2 ranks x 8 envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['config']['parallelism'], 'check', d['check']['ok'])"
timeout -k 10 600 python bench.py > $O/bench_noflags.json 2> $O/bench_noflags.err || { tail -20 $O/bench_noflags.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_noflags.json')); r=d['roofline']; print('no flags', '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'measured %.0f frac_measured %.4f' % (r['measured_peak'], r['frac_measured']), 'check', d['check']['ok'], 'cpu %.3e' % d['cpu_baseline']['value'], d['cpu_baseline']['kind'])"
