#!/bin/bash
# Round 6 final refresh, part 2: kernel traces (rocprofv3 --kernel-trace --stats) of the default bench (k_rollout,
# 64x64), 256x256 (k_rollout_bigq) and the MF-AC loop (k_acnet), then one FETCH_SIZE and one WRITE_SIZE pass per shape
# (one counter per pass), summarised into the build-keyed PMC files bench.py reads (summarize_prof.py stamps lib_sha16).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r06_final_b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof64 -o run --output-format csv -- python3 bench.py --steps 60 --warmup 8 --no-cpu-baseline --no-ceiling > $O/prof64.json 2> $O/prof64.err || exit 1
python3 scripts/timed_avg.py $O/prof64/run_kernel_trace.csv 3 > $O/timed_avg64.txt || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/f64 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-ceiling --check-envs 0 > $O/f64.json 2> $O/f64.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/w64 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-ceiling --check-envs 0 > $O/w64.json 2> $O/w64.err || exit 1
python3 scripts/summarize_prof.py $O/prof64 $O/f64 $O/w64 131072 $O/pmc_k_rollout.json 20 3 1 64 $O/prof64.json > /dev/null || exit 1
echo "pmc64 done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 80 --warmup 16 --no-cpu-baseline --no-ceiling > $O/prof256.json 2> $O/prof256.err || exit 1
python3 scripts/timed_avg.py $O/prof256/run_kernel_trace.csv 4 > $O/timed_avg256.txt || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/f256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 20 --warmup 16 --no-cpu-baseline --no-ceiling --check-envs 0 > $O/f256.json 2> $O/f256.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/w256 -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 20 --warmup 16 --no-cpu-baseline --no-ceiling --check-envs 0 > $O/w256.json 2> $O/w256.err || exit 1
python3 scripts/summarize_prof.py $O/prof256 $O/f256 $O/w256 2048 $O/pmc_big256.json 20 4 1 256 $O/prof256.json > /dev/null || exit 1
echo "pmc256 done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mfac -o run --output-format csv -- python3 bench.py --policy mfac --no-cpu-baseline --no-ceiling --steps 10 --warmup 2 > $O/prof_mfac.json 2> $O/prof_mfac.err || exit 1
python3 scripts/kernel_durations.py $O/prof_mfac/run_kernel_trace.csv k_acnet 20 > $O/kd_acnet.json || exit 1
rm -f $O/f64/run_counter_collection.csv $O/w64/run_counter_collection.csv $O/f256/run_counter_collection.csv $O/w256/run_counter_collection.csv $O/*/run_kernel_trace.csv
cp $O/pmc_k_rollout.json profiles/pmc_k_rollout.json
timeout -k 10 300 python bench.py > $O/bench_with_traffic.json 2> $O/bench_with_traffic.err || { tail -20 $O/bench_with_traffic.err; exit 1; }
cat $O/timed_avg64.txt $O/timed_avg256.txt $O/kd_acnet.json
python3 -c "import json; d=json.load(open('$O/bench_with_traffic.json')); r=d['roofline']; print('64x64', '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'frac_measured', r.get('frac_measured'), 'traffic', r.get('traffic'), r.get('traffic_is'))"
