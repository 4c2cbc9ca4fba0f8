# Round 3: same-box A/B of the Q-network forward kernels -- the previous form (build/libmagent_qold.so) against
# the software-pipelined LDS operand reads (build/libmagent.so): bench --policy qnet interleaved, then one
# kernel trace of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/qab}
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build
for r in 1 2; do
  for v in qold new; do
    if [ $v = qold ]; then export MAGENT_LIB=$L/libmagent_qold.so; else export MAGENT_LIB=$L/libmagent.so; fi
    timeout -k 10 300 python bench.py --policy qnet --steps 20 --warmup 3 --no-cpu-baseline > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$v', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'kernel_ms %.3f' % d['roofline']['kernel_ms'])"
  done
done
for v in qold new; do
  if [ $v = qold ]; then export MAGENT_LIB=$L/libmagent_qold.so; else export MAGENT_LIB=$L/libmagent.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --policy qnet --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_$v.json 2> $O/prof_$v.err || exit 1
  echo "== $v"; head -3 $O/prof_$v/run_kernel_stats.csv | cut -c1-160
done
