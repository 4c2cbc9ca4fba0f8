#!/bin/bash
# Round 6: where a per-call step of the generic configs goes -- kernel durations (rocprofv3 --kernel-trace --stats).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/da -o da -- python3 scripts/bench_generic.py --lib $L --config double_attack --map 24 --counts 40,60 --steps 200 > $O/da.log 2>&1 || { tail -5 $O/da.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fo -o fo -- python3 scripts/bench_generic.py --lib $L --config forest --map 32 --counts 60,50 --steps 200 > $O/fo.log 2>&1 || { tail -5 $O/fo.log; exit 1; }
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-6 $f | head -12; done
