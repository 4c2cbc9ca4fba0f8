set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/dropin_tests.log 2>&1 || { tail -40 gpurun_out/dropin_tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 200 python scripts/bench_dropin.py > gpurun_out/dropin.json 2> gpurun_out/dropin.err || exit 1
timeout -k 10 200 python scripts/bench_dropin.py --map 40 --agents 128 > gpurun_out/dropin40.json 2>> gpurun_out/dropin.err || exit 1
timeout -k 10 200 python scripts/bench_dropin.py --map 256 --agents 4096 > gpurun_out/dropin256.json 2>> gpurun_out/dropin.err || exit 1
