# Round 5: k_rollout over two halves on two streams (MFX_ROLLOUT_HALVES): parity, then 8192 / 16384 / 32768 envs A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05ag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "halves or substeps_match" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for C in "8192 1 0" "8192 2 0" "8192 2 4" "8192 2 8" "16384 1 0" "16384 2 0" "32768 1 0" "32768 2 0" "8192 1 0"; do
set -- $C; E=$1; H=$2; S=$3
MFX_ROLLOUT_HALVES=$H timeout -k 10 300 python bench.py --envs $E --substeps $S --no-cpu-baseline > $O/e.json 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/e.json')); r=d['roofline']; print('E=$E halves=$H S=%s %.4e frac %.4f ms/step %.4f check %s' % (d['config'].get('steps_per_launch'), d['value'], r['frac'], d['ms_per_step'], d.get('check', {}).get('ok')))"
done
