# 256x256: episode phases dealt round-robin over the two sub-batch pipelines (this build) against the
# contiguous deal (the previous build, kept as build/libmagent_prev.so); large-env parity tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_rollout_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --map 256 --agents 4096 --steps 40 --warmup 5 --no-cpu-baseline > $O/new_$r.json 2> $O/new_$r.err || exit 1
  MAGENT_LIB=$L/libmagent_prev.so timeout -k 10 200 python bench.py --map 256 --agents 4096 --steps 40 --warmup 5 --no-cpu-baseline > $O/prev_$r.json 2> $O/prev_$r.err || exit 1
  python3 -c "import json; a=json.load(open('$O/new_$r.json')); b=json.load(open('$O/prev_$r.json')); print('round-robin phases %.4g (frac %.3f)   contiguous %.4g (frac %.3f)' % (a['value'], a['roofline']['frac'], b['value'], b['roofline']['frac']))"
done
