# Round 5: env-chunked queue launches (MFX_BIGQ_CHUNK): parity tests, then 256x256 at 2048 / 3072 / 4096 envs chunked
# (the engine's choice) and in one launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05s}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "env_chunks or bigq_queue_step or bigq_bench_shape or reseed" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
for C in "3072 auto" "3072 0" "4096 auto" "4096 0" "2048 auto"; do
set -- $C; E=$1; K=$2
if [ $K = auto ]; then unset MFX_BIGQ_CHUNK; else export MFX_BIGQ_CHUNK=$K; fi
timeout -k 10 300 python bench.py --map 256 --agents 4096 --envs $E --substeps 20 --steps 60 --warmup 10 --check-envs 2 --no-cpu-baseline > $O/e${E}_$K.json 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/e${E}_$K.json')); r=d['roofline']; print('E=$E chunk=$K %.4e frac %.4f ms/step %.4f kernel_ms %.3f check %s' % (d['value'], r['frac'], d['ms_per_step'], r.get('kernel_ms', -1), d.get('check', {}).get('ok')))"
done
