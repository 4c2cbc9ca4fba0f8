# Round 3: (1) crossover of k_rollout vs the queue kernel for 64x64 batches (MFX_SMALL_E), (2) the 256x256
# bench at its 16-step default under rocprofv3 (kernel trace + FETCH_SIZE / WRITE_SIZE passes), (3) SQ
# wave-state counters of the current 4-step k_rollout.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03p
mkdir -p $O
export TMPDIR=/tmp
line() { python3 -c "import json;d=json.load(open('$1'));print('$2', d['config']['envs_per_gpu'], d['roofline']['kernel'], 'S', d['config']['steps_per_launch'], '%.4e'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'check', d['check']['ok'])"; }
for E in 128 256 512 1024 2048 4096 8192; do
  timeout -k 10 120 python bench.py --envs $E --steps 64 --warmup 16 --no-cpu-baseline > $O/kr_$E.json 2> $O/err || { tail -5 $O/err; exit 1; }
  line $O/kr_$E.json k_rollout
  MFX_SMALL_E=8192 MFX_BIGQ_ROWS=16 timeout -k 10 120 python bench.py --envs $E --substeps 16 --steps 64 --warmup 16 --no-cpu-baseline > $O/bq_$E.json 2> $O/err || { tail -5 $O/err; exit 1; }
  line $O/bq_$E.json "bigq R16"
done
for RS in "8 16" "16 32" "16 64"; do
  set -- $RS
  MFX_SMALL_E=64 MFX_BIGQ_ROWS=$1 timeout -k 10 120 python bench.py --total-envs 8 --substeps $2 --steps 192 --warmup 16 --no-cpu-baseline > $O/bq8_$1_$2.json 2> $O/err || { tail -5 $O/err; exit 1; }
  line $O/bq8_$1_$2.json "E=8 bigq R$1"
done
A="--map 256 --agents 4096 --steps 64 --warmup 16 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof256 -o run --output-format csv -- python3 bench.py $A > $O/prof256.json 2> $O/prof256.err || { tail -5 $O/prof256.err; exit 1; }
cat $O/prof256.json
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/f256 -o run --output-format csv -- python3 bench.py $A --check-envs 0 > $O/f256.json 2> $O/f256.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/w256 -o run --output-format csv -- python3 bench.py $A --check-envs 0 > $O/w256.json 2> $O/w256.err || exit 1
python3 scripts/summarize_prof.py $O/prof256 $O/f256 $O/w256 1024 $O/pmc_big256.json 16 4 4 256 $O/prof256.json > /dev/null || exit 1
python3 scripts/timed_avg.py $O/prof256/run_kernel_trace.csv 4 > $O/timed_avg256.txt; cat $O/timed_avg256.txt
rm -f $O/f256/run_counter_collection.csv.bak
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/sq -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --check-envs 0 > $O/sq.json 2> $O/sq.err || exit 1
python3 scripts/pmc_kernels.py $O/sq/run_counter_collection.csv SQ_WAVE_CYCLES 5 > $O/sq_wave.json
echo done
