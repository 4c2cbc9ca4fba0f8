# Round 5: k_acnet's image-staged GEMMs (direct-to-LDS weight chunks) A/B against the register staging, the policy
# parity tests, and the Ising scan's diagnostics.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_policy_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
for IMG in 0 1; do
MFX_ACNET_IMG=$IMG timeout -k 10 200 python scripts/bench_policy.py --net acnet > $O/acnet_img$IMG.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/acnet_img$IMG.json')); print('acnet img=$IMG ms %.3f tflops %.1f frac %.3f' % (d['ms_median'], d['tflops'], d['frac']))"
done
done
MFX_ISING_SCAN_STATS=1 timeout -k 10 200 python scripts/bench_ising.py --mode reference --no-cpu > $O/ising.json 2> $O/ising.err || { tail -20 $O/ising.err; exit 1; }
grep "ising scan" $O/ising.err | tail -2
