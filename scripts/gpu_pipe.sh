# Observation/step pipeline: rollout parity tests, then interleaved benches of the fused step
# (MFX_ROLLOUT_PIPE=0) against pipeline grid splits "step_per_cu:obs_per_cu".
#   scripts/gpu_pipe.sh "4:2 4:1 3:2" [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SPLITS=$1; shift
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rollout_gpu.py \
  > gpurun_out/pipe_tests.log 2>&1 || { tail -40 gpurun_out/pipe_tests.log; exit 1; }
tail -1 gpurun_out/pipe_tests.log
for r in 1 2; do for v in fused $SPLITS; do
if [ $v = fused ]; then export MFX_ROLLOUT_PIPE=0; else export MFX_ROLLOUT_PIPE=1 MFX_PIPE_STEP_PER_CU=${v%:*} MFX_PIPE_OBS_PER_CU=${v#*:}; fi
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/pipe_${v/:/_}_$r.json 2> gpurun_out/pipe.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/pipe_${v/:/_}_$r.json')); print('$v', $r, '%.4e' % d['value'], 'ms %.4f' % d['ms_per_step'], 'kernel %.4f' % d['roofline']['kernel_ms'])"
done; done
