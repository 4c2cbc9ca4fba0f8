# Round 2: kernel trace of the fast drop-in path (k_dropin_step durations) at 40x40 and 64x64
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02
export TMPDIR=/tmp
O=gpurun_out/r02
for m in "40 128" "64 256"; do
  set -- $m
  MFX_DROPIN_FAST=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_dropin$1 -o run --output-format csv -- python3 scripts/bench_dropin.py --map $1 --agents $2 --seconds 3 > $O/prof_dropin$1.json 2> $O/prof_dropin$1.err || exit 1
done
