# Round 3: the GPU suite and smoke on the current tree, then the Q-net kernel A/B and the 256x256 substeps sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/c3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --durations=15 --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash scripts/gpu_r03_qnet_vec.sh && bash scripts/gpu_r03_sub256.sh
