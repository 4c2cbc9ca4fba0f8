# Round 5 final refresh of the committed tree: the whole GPU suite, smoke, the bench lines (default with the 16-process
# CPU baseline, 256x256, configs[3] shapes, the 2-rank gloo rehearsal, the learned MF-Q and MFAC policies), kernel
# traces and FETCH_SIZE / WRITE_SIZE passes of k_rollout (64x64) and k_rollout_bigq (256x256), one counter per pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05z_final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --durations=15 --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('64x64', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'], 'cpu', '%.3e' % d['cpu_baseline']['value'])"
timeout -k 10 400 python bench.py --map 256 --agents 4096 --steps 20 --warmup 5 > $O/bench256.json 2> $O/bench256.err || { tail -20 $O/bench256.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench256.json')); print('256x256', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'], 'cpu', '%.3e' % d['cpu_baseline']['value'])"
for E in 8 64 8192; do
timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/bench_${E}envs.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_${E}envs.json')); print('$E envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'frac %.4f' % d['roofline']['frac'], 'S', d['config']['steps_per_launch'], 'check', d['check']['ok'])"
done
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --envs 2048 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_2rank.json 2> $O/bench_2rank.err || { tail -20 $O/bench_2rank.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2rank.json')); print('2 ranks', d['n_gpus'], d['ranks'], d['config']['parallelism'], d['episodes']['note'])"
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --total-envs 16 --steps 256 --warmup 64 --no-cpu-baseline > $O/bench_2rank_16envs.json 2> $O/bench_2rank_16envs.err || { tail -20 $O/bench_2rank_16envs.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2rank_16envs.json')); print('2 ranks x 8 envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['config']['parallelism'], 'check', d['check']['ok'])"
timeout -k 10 400 python bench.py --map 256 --agents 4096 --envs 4096 --steps 40 --warmup 10 --no-cpu-baseline > $O/bench256_4096.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench256_4096.json')); print('256x256 4096 envs', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
timeout -k 10 400 python scripts/bench_ising.py --mode reference > $O/ising_reference.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/ising_reference.json')); print('ising reference', d['replicas'], '%.4e' % d['value'], d['check'])"
timeout -k 10 300 python scripts/bench_ising.py --mode philox --no-cpu > $O/ising_philox.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/ising_philox.json')); print('ising philox', d['replicas'], '%.4e' % d['value'])"
timeout -k 10 200 python scripts/bench_dropin.py --map 40 --agents 128 --seconds 4 --calls > $O/dropin_40.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/dropin_40.json')); print('drop-in 40x40 vs ref', '%.3f' % d['hip_vs_ref'])"
for P in qnet mfac; do
timeout -k 10 300 python bench.py --policy $P --no-cpu-baseline > $O/bench_$P.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_$P.json')); print('$P', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'])"
done
for N in acnet qnet; do
timeout -k 10 200 python scripts/bench_policy.py --net $N > $O/fwd_$N.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/fwd_$N.json')); print('$N forward frac %.3f' % d['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mfac -o run --output-format csv -- python3 bench.py --policy mfac --no-cpu-baseline --steps 10 --warmup 2 > $O/prof_mfac.json 2> $O/prof_mfac.err || exit 1
python3 scripts/kernel_durations.py $O/prof_mfac/run_kernel_trace.csv k_acnet 20 > $O/kd_acnet.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof64 -o run --output-format csv -- python3 bench.py --steps 60 --warmup 8 --no-cpu-baseline > $O/prof64.json 2> $O/prof64.err || exit 1
python3 scripts/timed_avg.py $O/prof64/run_kernel_trace.csv 3 > $O/timed_avg64.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 80 --warmup 16 --no-cpu-baseline > $O/prof256.json 2> $O/prof256.err || exit 1
python3 scripts/timed_avg.py $O/prof256/run_kernel_trace.csv 4 > $O/timed_avg256.txt || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/f64 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --check-envs 0 > $O/f64.json 2> $O/f64.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/w64 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --check-envs 0 > $O/w64.json 2> $O/w64.err || exit 1
python3 scripts/summarize_prof.py $O/prof64 $O/f64 $O/w64 131072 $O/pmc_k_rollout.json 20 3 1 64 $O/prof64.json > /dev/null || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/f256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 20 --warmup 16 --no-cpu-baseline --check-envs 0 > $O/f256.json 2> $O/f256.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/w256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 20 --warmup 16 --no-cpu-baseline --check-envs 0 > $O/w256.json 2> $O/w256.err || exit 1
python3 scripts/summarize_prof.py $O/prof256 $O/f256 $O/w256 2048 $O/pmc_big256.json 20 4 1 256 $O/prof256.json > /dev/null || exit 1
rm -f $O/f64/run_counter_collection.csv $O/w64/run_counter_collection.csv $O/f256/run_counter_collection.csv $O/w256/run_counter_collection.csv
cat $O/timed_avg64.txt $O/timed_avg256.txt $O/kd_acnet.json
