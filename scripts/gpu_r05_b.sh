# Round 5: the headline kernel against the reference recording (battle64_rollout), the row movers' index fixes,
# and the default bench line with its reference-build check.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py tests/test_replay_gpu.py tests/test_algo_gpu.py \
  -k "reference_recording or rows_copy or replay or algo" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); c=d['check']; print('64x64', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', c['ok'], 'ref env', c['reference_env_rank0'], c['reference_envs'], 'cpu', '%.3e' % d['cpu_baseline']['value'])"
