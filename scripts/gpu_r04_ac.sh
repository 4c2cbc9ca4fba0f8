# Round 4: the heavy (workgroup-team) steps file their items beside the policy loop -- rollout tests, stamps, configs[3].
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04ac}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rollout_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
MAGENT_LIB=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 200 \
    python scripts/stamps_few.py --envs 8 > $O/stamps_8.txt 2>&1 || { tail -20 $O/stamps_8.txt; exit 1; }
grep -E "pipelined|agents:" $O/stamps_8.txt | cut -c1-300
for rep in 1 2; do for K in 60 256; do for E in 8 64; do
  timeout -k 10 200 python bench.py --total-envs $E --steps $K --warmup 64 --no-cpu-baseline > $O/e${E}_k${K}_$rep.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_k${K}_$rep.json
done; done; done
