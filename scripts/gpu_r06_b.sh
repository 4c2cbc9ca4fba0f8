# Round 6: MFAC loop -- the view layer over the engine's view support, and env batches on two streams.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r06b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_policy_gpu.py -k "acnet or mfac" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for V in "--dense-view" "" "--split 2" "--split 2 --envs 16384" "--split 4 --envs 16384"; do
N=$(echo "$V" | tr -d ' -')
timeout -k 10 300 python bench.py --policy mfac --no-cpu-baseline $V > $O/mfac_$N.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/mfac_$N.json')); r=d['roofline']; print('mfac [$V]', '%.4e' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'fwd %.3f env %.3f' % (r['kernel_ms'], r['env_step_ms']), 'frac %.4f' % r['frac'], 'views', d['config']['view_inputs'])"
done
