# Drop-in resident server: actions in the mailbox poll (MFX_DROPIN_MAIL=1) vs header-only poll + one
# action round trip (MFX_DROPIN_MAIL=0), interleaved, 40x40 and 64x64.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_battle_gpu.py -k "dropin or replays_reference_fixture" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for m in 1 0; do
    for mp in "40 128" "64 256"; do
      set -- $mp
      MFX_DROPIN_MAIL=$m timeout -k 10 120 python scripts/bench_dropin.py --map $1 --agents $2 --seconds 4 > $O/m${m}_$1_$r.json 2>> $O/bench.err || exit 1
      python3 -c "import json; d=json.load(open('$O/m${m}_$1_$r.json')); print('mail=$m map=$1', '%.4g'%d['hip_dropin'], 'C %.4g'%d['c_oracle_1thread'], '%.3f'%(d['hip_dropin']/d['c_oracle_1thread']))"
    done
  done
done
