# Round 4: the drop-in's one-call getters (mfx_env_get_rows) -- the drop-in / ABI tests, then the drop-in against the
# reference engine itself (oracle/_ref, one thread) and the C oracle, 40x40 and 64x64.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04u}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_abi_trace.py tests/test_battle_gpu.py tests/test_algo_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for m in "40 128" "64 256"; do set -- $m
  timeout -k 10 200 python scripts/bench_dropin.py --map $1 --agents $2 --seconds 4 --calls > $O/dropin_$1.json 2> $O/err || { tail -20 $O/err; exit 1; }
  cat $O/dropin_$1.json
done; done
