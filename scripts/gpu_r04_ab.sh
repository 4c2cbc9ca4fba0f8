# Round 4: bench.py timing the region with one event pair (not a pair per launch) -- 8192 envs (128 launches of 2
# steps), the default, configs[3]; a rocprofv3 kernel trace of the 8192-env run to check kernel_ms.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04ab}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 200 python bench.py --total-envs 8192 --steps 256 --warmup 16 --no-cpu-baseline > $O/e8192_$rep.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'ms/step %.4f' % d['ms_per_step'], 'kernel_ms %.4f' % r['kernel_ms'], d['check']['ok'])" $O/e8192_$rep.json
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/def.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'ms/step %.4f' % d['ms_per_step'], 'kernel_ms %.4f' % r['kernel_ms'], d['check']['ok'])" $O/def.json
timeout -k 10 200 python bench.py --total-envs 8 --steps 256 --warmup 64 --no-cpu-baseline > $O/e8.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'kernel_ms %.4f' % r['kernel_ms'], d['check']['ok'])" $O/e8.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8192 -o run --output-format csv -- python3 bench.py --total-envs 8192 --steps 256 --warmup 16 --no-cpu-baseline > $O/prof8192.json 2> $O/prof8192.err || exit 1
python3 scripts/timed_avg.py $O/prof8192/run_kernel_trace.csv 128 > $O/timed_avg8192.txt || exit 1
cat $O/timed_avg8192.txt
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('profiled', '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'kernel_ms %.4f' % r['kernel_ms'])" $O/prof8192.json
