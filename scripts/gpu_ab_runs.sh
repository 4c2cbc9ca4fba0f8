set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py tests/test_battle_gpu.py > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
for r in 1 2; do for V in libmagent libmagent_noruns; do
MAGENT_LIB=$L/$V.so timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/ab64_${V}_$r.json 2> gpurun_out/ab.err || exit 1
MAGENT_LIB=$L/$V.so timeout -k 10 300 python bench.py --map 256 --agents 4096 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab256_${V}_$r.json 2> gpurun_out/ab.err || exit 1
done; done
