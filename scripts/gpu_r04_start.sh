# Round 4, first box: the new reference-pinned 256x256 tests (full episodes through the per-call ABI,
# k_rollout_bigq against the reference recording and the reference build), then the batch-size sweep of
# k_rollout at 20 steps per launch (8192 / 32768 / 131072 envs, S=4 at 8192 for the round-3 comparison).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04s}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --durations=10 --timeout 300 --timeout-method thread -m gpu \
  "tests/test_battle_gpu.py::test_hip_replays_reference_large_map" \
  "tests/test_rollout_gpu.py::test_rollout_bigq_matches_reference_recording" \
  "tests/test_rollout_gpu.py::test_rollout_bigq_bench_shape_matches_reference_build" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for E in 8192 32768 131072; do
timeout -k 10 300 python bench.py --envs $E --steps 60 --warmup 10 --no-cpu-baseline --check-envs 2 > $O/e${E}_s20.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['roofline']['frac'], d['ms_per_step'], d['check']['ok'])" $O/e${E}_s20.json
done
timeout -k 10 300 python bench.py --envs 8192 --substeps 4 --steps 60 --warmup 10 --no-cpu-baseline --check-envs 2 > $O/e8192_s4.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['roofline']['frac'], d['ms_per_step'], d['check']['ok'])" $O/e8192_s4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8k -o run --output-format csv -- python3 bench.py --envs 8192 --steps 60 --warmup 10 --no-cpu-baseline --check-envs 0 > $O/prof8k.json 2> $O/prof8k.err || exit 1
python3 scripts/timed_avg.py $O/prof8k/run_kernel_trace.csv 3 > $O/timed_avg8k.txt || exit 1
cat $O/timed_avg8k.txt
