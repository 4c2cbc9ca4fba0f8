# Round 5: k_acnet layers chained (each layer's last chunk issues the next one's first): tests, forward, MFAC loop.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05ah}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_policy_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2 3; do
timeout -k 10 200 python scripts/bench_policy.py --net acnet > $O/acnet$k.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/acnet$k.json')); print('acnet ms %.3f tflops %.1f frac %.3f' % (d['ms_median'], d['tflops'], d['frac']))"
done
timeout -k 10 400 python bench.py --policy mfac --no-cpu-baseline > $O/bench_mfac.json 2> $O/bench_mfac.err || { tail -20 $O/bench_mfac.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_mfac.json')); r=d['roofline']; print('mfac value %.4e ms/step %.3f' % (d['value'], d['ms_per_step']), r['frac'], r['kernel_ms'])"
