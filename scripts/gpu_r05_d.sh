# Round 5: the learned-policy forwards alone (scripts/bench_policy.py) and their SQ counters: where k_acnet and the
# QNet kernels lose against the f32 MFMA peak.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05d}
mkdir -p $O
export TMPDIR=/tmp
for NET in acnet qnet; do
timeout -k 10 200 python scripts/bench_policy.py --net $NET > $O/bench_$NET.json 2> $O/err || { tail -20 $O/err; exit 1; }
cat $O/bench_$NET.json
done
cd /tmp
P=$GRAFT_REPO_ROOT/$O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $P/pmc1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_policy.py --net acnet --reps 3 > $P/pmc1.json 2> $P/pmc1.err || { tail -20 $P/pmc1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $P/pmc2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_policy.py --net acnet --reps 3 > $P/pmc2.json 2> $P/pmc2.err || { tail -20 $P/pmc2.err; exit 1; }
find $P -name "*counter_collection.csv" | head
