# Round 4: steps per launch (--substeps) at small batches -- 8 and 64 envs (pipelined few-env path), 8192 and 32768
# envs (k_rollout), two interleaved reps, every line self-checked.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04o}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for E in 8192 32768; do for S in 2 4 5 8 20; do
    timeout -k 10 200 python bench.py --total-envs $E --substeps $S --steps 80 --warmup 16 --no-cpu-baseline > $O/e${E}_s$S.json 2> $O/err || { tail -20 $O/err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_s$S.json
  done; done
  for E in 8 64; do for S in 5 10 20 40; do
    timeout -k 10 200 python bench.py --total-envs $E --substeps $S --steps 200 --warmup 40 --no-cpu-baseline > $O/e${E}_s$S.json 2> $O/err || { tail -20 $O/err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_s$S.json
  done; done
done
