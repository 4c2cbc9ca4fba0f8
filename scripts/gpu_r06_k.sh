#!/bin/bash
# Round 6: per-shape workgroups per CU, no division for the shifted row: parity, default vs 2 and 3 per CU.
set -o pipefail
mkdir -p gpurun_out/r06k
B=mean-field-multi-agent-reinforcement-learning_amd/build
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_replay_gpu.py tests/test_algo_gpu.py \
  > gpurun_out/r06k/tests.log 2>&1 && tail -1 gpurun_out/r06k/tests.log || exit 1
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1].split('/')[-1], '%.4e'%d['value'], '%.4f'%d['roofline']['frac'])" $1; }
for r in 1 2; do
  timeout -k 10 120 python -u scripts/bench_replay.py --cpu-seconds 1 > gpurun_out/r06k/fusedD_$r.json && show gpurun_out/r06k/fusedD_$r.json || exit 1
  timeout -k 10 120 python -u scripts/bench_replay.py --cpu-seconds 1 --two-launches > gpurun_out/r06k/twoD_$r.json && show gpurun_out/r06k/twoD_$r.json || exit 1
  for n in 2 3; do
    MAGENT_LIB=$B/libmagent_rows$n.so timeout -k 10 120 python -u scripts/bench_replay.py --cpu-seconds 1 > gpurun_out/r06k/fused${n}_$r.json && show gpurun_out/r06k/fused${n}_$r.json || exit 1
    MAGENT_LIB=$B/libmagent_rows$n.so timeout -k 10 120 python -u scripts/bench_replay.py --cpu-seconds 1 --two-launches > gpurun_out/r06k/two${n}_$r.json && show gpurun_out/r06k/two${n}_$r.json || exit 1
  done
done
