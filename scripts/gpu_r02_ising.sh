# Round 2: Ising tests (multi-episode, large lattices) and the drop-in after the LDS RolloutArgs change
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ising_gpu.py tests/test_battle_gpu.py -k "ising or episodes or lattice or odd_call or replays_reference_fixture or philox or dropin or reference_loop" > $O/ising_tests.log 2>&1 || { tail -40 $O/ising_tests.log; exit 1; }
timeout -k 10 120 python scripts/bench_ising.py > $O/bench_ising.json 2> $O/bench_ising.err || exit 1
