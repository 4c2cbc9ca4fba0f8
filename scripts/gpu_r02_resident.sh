# Round 2: the resident drop-in server (one k_dropin_step launch answering every env.step() through a
# mailbox in coherent host memory) -- drop-in parity tests, then timing against the one-shot launch
# per step (MFX_DROPIN_RESIDENT=0), the per-call path (MFX_DROPIN_FAST=0) and the C oracle.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_battle_gpu.py tests/test_abi_trace.py tests/test_rules_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in "40 128" "64 256"; do
  set -- $m
  timeout -k 10 120 python scripts/bench_dropin.py --map $1 --agents $2 --calls > $O/res_$1.json 2>> $O/bench.err || exit 1
  MFX_DROPIN_RESIDENT=0 timeout -k 10 120 python scripts/bench_dropin.py --map $1 --agents $2 --calls > $O/oneshot_$1.json 2>> $O/bench.err || exit 1
  cat $O/res_$1.json $O/oneshot_$1.json
done
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so
MAGENT_LIB=$L timeout -k 10 120 python scripts/stamps_dropin.py --map 40 --agents 128 > $O/stamps40.txt 2>&1 || { cat $O/stamps40.txt; exit 1; }
MAGENT_LIB=$L timeout -k 10 120 python scripts/stamps_dropin.py --map 64 --agents 256 > $O/stamps64.txt 2>&1 || { cat $O/stamps64.txt; exit 1; }
grep map $O/stamps40.txt $O/stamps64.txt
