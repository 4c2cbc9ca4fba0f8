# Round 2: launcher rehearsal, configs[3], lanes A/B (interleaved), multi-core CPU baseline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02
export TMPDIR=/tmp
O=gpurun_out/r02
nproc > $O/nproc.txt; python -c "import os; print(len(os.sched_getaffinity(0)), os.environ.get('OMP_NUM_THREADS'))" >> $O/nproc.txt
for i in 1 2; do
  for L in 1 2 3; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --lanes $L >> $O/lanes.jsonl 2>> $O/lanes.err || exit 1
  done
done
timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs 64 > $O/cfg3_1gpu.json 2> $O/cfg3.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --gpus 2 --backend gloo --envs 4096 > $O/launch2.json 2> $O/launch2.err || exit 1
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --total-envs 64 --no-cpu-baseline > $O/launch2_cfg3.json 2> $O/launch2_cfg3.err || exit 1
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
