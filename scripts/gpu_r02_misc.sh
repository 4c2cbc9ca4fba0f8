# Round 2: launch round-trip floor, the reference-wrapper ABI trace on libmagent.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02
export TMPDIR=/tmp
O=gpurun_out/r02
timeout -k 10 120 ./scripts/micro/launch_rtt > $O/launch_rtt.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_abi_trace.py tests/test_mf.py tests/test_algo_gpu.py -k "reference or kernel or replay" > $O/abi_tests.log 2>&1 || { tail -30 $O/abi_tests.log; exit 1; }
