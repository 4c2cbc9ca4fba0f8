# Round 4: the drop-in single env against the reference engine itself (oracle/_ref, one thread) and the C oracle,
# 40x40 and 64x64, per-call times.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04t}
mkdir -p $O
export TMPDIR=/tmp
for m in "40 128" "64 256"; do set -- $m
  timeout -k 10 200 python scripts/bench_dropin.py --map $1 --agents $2 --seconds 4 --calls > $O/dropin_$1.json 2> $O/err || { tail -20 $O/err; exit 1; }
  cat $O/dropin_$1.json
done
