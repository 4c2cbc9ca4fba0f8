# Rollout parity tests under a library variant, then an interleaved A/B bench:
#   scripts/gpu_variant_check.sh "V1 V2 ..." [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
VS=$1; shift
for v in $VS; do
MAGENT_LIB=$L/libmagent_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_rollout_gpu.py > gpurun_out/vc_tests_$v.log 2>&1 || { tail -30 gpurun_out/vc_tests_$v.log; exit 1; }
tail -1 gpurun_out/vc_tests_$v.log
done
bash scripts/gpu_ab_multi.sh "$VS" "$@"
