# Round 4: is the stepper slowed by the item workers sharing its CU?  Grid 512 (two workgroups per CU) vs 256.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04y}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do for G in 0 256; do for E in 8 64; do
  MFX_BIGQ_GRID=$G timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/e${E}_g$G.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_g$G.json
done; done; done
for G in 0 256; do
  MFX_BIGQ_GRID=$G MAGENT_LIB=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 200 \
      python scripts/stamps_few.py --envs 8 > $O/stamps_g$G.txt 2>&1 || { tail -20 $O/stamps_g$G.txt; exit 1; }
  echo "== grid $G"; grep -E "pipelined|agents:" $O/stamps_g$G.txt | cut -c1-300
done
