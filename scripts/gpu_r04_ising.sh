# Round 4: measurement evidence for the Ising kernels at configs[0]'s shape (20x20, tau 0.8): k_ising_mfq in
# reference mode (host numpy streams, bit-exact) and Philox mode -- bench lines with both CPU baselines, kernel
# traces, FETCH_SIZE / WRITE_SIZE passes and one SQ wave-state pass per mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04is}
mkdir -p $O
export TMPDIR=/tmp
for M in reference philox; do
  S=2000; [ $M = reference ] && S=1000
  timeout -k 10 300 python scripts/bench_ising.py --mode $M --steps $S > $O/bench_$M.json 2> $O/err || { tail -20 $O/err; exit 1; }
  cat $O/bench_$M.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$M -o run --output-format csv -- python3 scripts/bench_ising.py --mode $M --steps $S --no-cpu > $O/tr_$M.json 2> $O/tr_$M.err || exit 1
  python3 scripts/kernel_durations.py $O/tr_$M/run_kernel_trace.csv k_ising_mfq > $O/kd_$M.json || exit 1
  cat $O/kd_$M.json
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f_$M -o run --output-format csv -- python3 scripts/bench_ising.py --mode $M --steps $S --no-cpu > /dev/null 2> $O/f_$M.err || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_$M -o run --output-format csv -- python3 scripts/bench_ising.py --mode $M --steps $S --no-cpu > /dev/null 2> $O/w_$M.err || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/sq_$M -o run --output-format csv -- python3 scripts/bench_ising.py --mode $M --steps $S --no-cpu > /dev/null 2> $O/sq_$M.err || exit 1
  python3 scripts/sq_summary.py $O/sq_$M/run_counter_collection.csv 1 "k_ising_mfq $M mode" k_ising_mfq > $O/sq_$M.json || exit 1
  python3 scripts/pmc_kernel_bytes.py $O/f_$M/run_counter_collection.csv $O/w_$M/run_counter_collection.csv k_ising_mfq > $O/pmc_$M.json || exit 1
  cat $O/pmc_$M.json
done
