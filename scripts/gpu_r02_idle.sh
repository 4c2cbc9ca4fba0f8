# Drop-in resident server when the caller's policy takes longer than the idle timeout between steps
# (the server leaves and is relaunched every step): env.step() time with a 3 ms host pause per step,
# resident vs one launch per step; then the drop-in GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_battle_gpu.py -k "dropin or replays_reference_fixture" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python scripts/bench_dropin.py --map 40 --agents 128 --seconds 0.08 --calls --pause-us 3000 > $O/res_pause.json 2>> $O/bench.err || exit 1
MFX_DROPIN_RESIDENT=0 timeout -k 10 120 python scripts/bench_dropin.py --map 40 --agents 128 --seconds 0.08 --calls --pause-us 3000 > $O/oneshot_pause.json 2>> $O/bench.err || exit 1
python3 -c "
import json
for f in ('res_pause','oneshot_pause'):
    d=json.load(open('$O/'+f+'.json')); print(f, 'step us', d['us_per_step']['hip_dropin']['step'], 'agent-steps/s (timed calls only) %.4g' % d['hip_dropin'])
"
