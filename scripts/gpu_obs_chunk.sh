set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for R in 64 128; do for K in 2 3; do for D in 4 6 8; do
MFX_ITEM_ROWS=$R MFX_BIG_SPLIT=$K MFX_ITEM_GRID_DIV=$D timeout -k 10 300 python bench.py --map 256 --agents 4096 --envs 1024 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/items_r${R}_k${K}_d$D.json 2> gpurun_out/items.err || exit 1
done; done; done
