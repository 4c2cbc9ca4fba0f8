# Round 3: same-box A/B of the Q-network conv kernel's LDS read scheduling: the previous form (qold), conv1's
# next-tile prefetch only (qc1), conv2's next-k-step prefetch only (qc2), both (new); kernel traces, two rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/qab2}
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build
for r in 1 2; do
  for v in qold qc1 qc2 new; do
    if [ $v = new ]; then export MAGENT_LIB=$L/libmagent.so; else export MAGENT_LIB=$L/libmagent_$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${v}_$r -o run --output-format csv -- python3 bench.py --policy qnet --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_${v}_$r.json 2> $O/prof_${v}_$r.err || exit 1
    python3 -c "
import csv
for x in csv.DictReader(open('$O/prof_${v}_$r/run_kernel_stats.csv')):
    if 'qnet_conv' in x['Name'] or 'qnet_head' in x['Name']: print('$v r$r', x['Name'][5:20], '%.3f ms' % (float(x['AverageNs']) / 1e6))
"
    rm -f $O/prof_${v}_$r/run_kernel_trace.csv
  done
done
