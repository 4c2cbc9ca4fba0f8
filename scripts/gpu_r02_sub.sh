# Round 2: substeps parity (new tests), then the substeps sweep (interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02
export TMPDIR=/tmp
O=gpurun_out/r02
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rollout_gpu.py -k "substeps or bench_shape" > $O/sub_tests.log 2>&1 || { tail -30 $O/sub_tests.log; exit 1; }
for i in 1 2; do
  for S in 1 2 4 8 16; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --substeps $S --steps 64 >> $O/sub_sweep.jsonl 2>> $O/sub_sweep.err || exit 1
  done
done
