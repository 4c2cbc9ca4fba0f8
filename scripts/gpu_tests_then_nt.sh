# GPU tests, then HBM ceilings and the A/B of nontemporal obs stores
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
bash scripts/gpu_nt_ab.sh
