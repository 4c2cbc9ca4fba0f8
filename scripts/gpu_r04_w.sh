# Round 4: queue-kernel launches serialised process-wide (BigqSerial) -- two engines on two streams, and the few-env /
# large-env rollout tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04w}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "two_engines|passed|failed" $O/tests.log | tail -4
timeout -k 10 200 python bench.py --total-envs 8 --steps 256 --warmup 64 --no-cpu-baseline > $O/e8.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/e8.json')); print('8 envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'check', d['check']['ok'])"
timeout -k 10 400 python bench.py --map 256 --agents 4096 --steps 20 --warmup 5 --no-cpu-baseline > $O/b256.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b256.json')); print('256', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
