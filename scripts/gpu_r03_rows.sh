# Round 3: measurement of the other 8 rows -- the replay data path (k_rows_copy) and the Ising MF-Q kernel --
# each next to its CPU baseline.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03rows
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python scripts/bench_replay.py > $O/replay.json 2> $O/replay.err || { tail -20 $O/replay.err; exit 1; }
cat $O/replay.json
timeout -k 10 200 python scripts/bench_ising.py --replicas 16384 > $O/ising.json 2> $O/ising.err || { tail -20 $O/ising.err; exit 1; }
cat $O/ising.json
