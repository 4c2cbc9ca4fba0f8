# WRITE_SIZE / FETCH_SIZE per launch against steps per launch (1, 2, 4): is the extra traffic real?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02/pmcsub
mkdir -p $O
export TMPDIR=/tmp
for S in 1 2 4; do
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w$S -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --substeps $S --no-cpu-baseline > $O/w$S.json 2> $O/w$S.err || exit 1
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f$S -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --substeps $S --no-cpu-baseline > $O/f$S.json 2> $O/f$S.err || exit 1
done
