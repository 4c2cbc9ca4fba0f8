# Round 5: the queue kernels' forward progress without co-residency (stepper claims, stolen items, per-XCD exit):
# the few-env / queue-kernel rollout tests, the 2-rank shared-card rehearsal of configs[3] on the pipelined path, and
# the 8 / 64-env lines (no regression of the pipelined stepper).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py \
  -k "one_workgroup or few_pipe or two_engines or small_e or bigq_matches_reference or substeps_auto" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --total-envs 16 --steps 256 --warmup 64 --no-cpu-baseline > $O/bench_2rank_16envs.json 2> $O/e2.err || { tail -20 $O/e2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2rank_16envs.json')); print('2 ranks x 8 envs', '%.4e' % d['value'], d['config']['workload'], 'kernel', d['roofline']['kernel'], 'check', d['check']['ok'], d['check']['path'])"
for E in 8 64; do
timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/bench_${E}envs.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_${E}envs.json')); print('$E envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'frac %.4f' % d['roofline']['frac'], 'S', d['config']['steps_per_launch'], 'check', d['check']['ok'])"
done
