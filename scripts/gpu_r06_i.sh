#!/bin/bash
# Round 6: fused replay sample (current + next-state columns in one launch) -- parity, then A/B against two launches.
set -o pipefail
mkdir -p gpurun_out/r06i
export PYTHONPATH=$PWD/mean-field-multi-agent-reinforcement-learning_amd/python
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_replay_gpu.py tests/test_algo_gpu.py \
  > gpurun_out/r06i/tests.log 2>&1 && tail -1 gpurun_out/r06i/tests.log &&
for r in 1 2; do
  timeout -k 10 120 python -u scripts/bench_replay.py --cpu-seconds 1 > gpurun_out/r06i/fused_$r.json &&
  timeout -k 10 120 python -u scripts/bench_replay.py --cpu-seconds 1 --two-launches > gpurun_out/r06i/two_$r.json || exit 1
  python -c "import json;[print(n, '%.4e'%d['value'], '%.4f'%d['roofline']['frac'], d['ms_per_sample_median']) for n in ['fused_$r','two_$r'] for d in [json.load(open('gpurun_out/r06i/'+n+'.json'))]]"
done
