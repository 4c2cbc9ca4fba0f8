# Round 4: the pipelined form on one workgroup per CU by default -- rollout tests, configs[3] shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04aa}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for K in 256 1024; do for E in 8 64; do
  timeout -k 10 200 python bench.py --total-envs $E --steps $K --warmup 64 --no-cpu-baseline > $O/e${E}_k$K.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'grid', d['roofline']['grid'], d['check']['ok'])" $O/e${E}_k$K.json
done; done; done
