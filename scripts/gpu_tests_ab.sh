# GPU tests on the default build, then an A/B of library variants (two rounds): scripts/gpu_tests_ab.sh v1 v2 ...
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash scripts/gpu_variants.sh "$@" "$@"
