# Round 3: the Battle observation stream with the per-cell offset table and division-free stream
# positions -- rollout parity tests on the new library, then an interleaved A/B of the default bench
# against the previous library (build/libmagent_prev.so) or the libraries named in $LIBS.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03obs
mkdir -p $O
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_rollout_gpu.py > $O/tests_rollout.log 2>&1 || { tail -40 $O/tests_rollout.log; exit 1; }
grep -E "passed|failed" $O/tests_rollout.log | tail -1
for r in 1 2 3; do for lib in ${LIBS:-libmagent libmagent_prev}; do
MAGENT_LIB=$L/$lib.so timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/ab_${lib}_$r.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
python -c "import json; d=json.load(open('$O/ab_${lib}_$r.json')); r=d['roofline']; print('$lib', $r, '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'kms %.4f' % r['kernel_ms'], 'lds', r['lds_bytes'], 'grid', r['grid'], 'check', d['check']['ok'])"
done; done
