#!/bin/bash
# Round 6: k_rows_pipe rows in flight per wave -- parity on the product build, then depth 2 (product) vs 3 vs 4.
set -o pipefail
mkdir -p gpurun_out/r06l
B=mean-field-multi-agent-reinforcement-learning_amd/build
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_replay_gpu.py tests/test_algo_gpu.py \
  > gpurun_out/r06l/tests.log 2>&1 && tail -1 gpurun_out/r06l/tests.log || exit 1
MAGENT_LIB=$B/libmagent_d3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_replay_gpu.py \
  > gpurun_out/r06l/tests_d3.log 2>&1 && tail -1 gpurun_out/r06l/tests_d3.log || exit 1
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1].split('/')[-1], '%.4e'%d['value'], '%.4f'%d['roofline']['frac'])" $1; }
for r in 1 2; do
  for v in magent magent_d3 magent_d4 magent_d4cu1; do
    MAGENT_LIB=$B/lib$v.so timeout -k 10 120 python -u scripts/bench_replay.py --cpu-seconds 1 > gpurun_out/r06l/fused_${v}_$r.json && show gpurun_out/r06l/fused_${v}_$r.json || exit 1
    MAGENT_LIB=$B/lib$v.so timeout -k 10 120 python -u scripts/bench_replay.py --cpu-seconds 1 --two-launches > gpurun_out/r06l/two_${v}_$r.json && show gpurun_out/r06l/two_${v}_$r.json || exit 1
  done
done
