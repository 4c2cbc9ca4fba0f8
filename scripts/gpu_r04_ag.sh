# Round 4: replay mover workgroups per CU (k_rows_pipe), 3-6, two interleaved reps.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04ag}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do for W in 3 4 5 6 8; do
  MFX_ROWS_WG_PER_CU=$W timeout -k 10 200 python scripts/bench_replay.py --cpu-seconds 0.5 > $O/w$W.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e rows/s' % d['value'], 'frac %.4f' % d['roofline']['frac'])" $O/w$W.json
done; done
