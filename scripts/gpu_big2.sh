set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in 512 1024 2048; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_big_E$E -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --envs $E --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_big_E$E.json 2> gpurun_out/prof_big.err || exit 1
python scripts/sum_big.py gpurun_out/prof_big_E$E
done
