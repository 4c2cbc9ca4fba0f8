# Round 4: steps per launch, finer: 8192 envs S = 1-3, 16384 envs S = 2-20, few envs S = 40 / 64.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04p}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for V in "8192 1" "8192 2" "8192 3" "8192 20" "16384 2" "16384 4" "16384 8" "16384 20"; do set -- $V
    timeout -k 10 200 python bench.py --total-envs $1 --substeps $2 --steps 80 --warmup 16 --no-cpu-baseline > $O/e$1_s$2.json 2> $O/err || { tail -20 $O/err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/e$1_s$2.json
  done
  for V in "8 40" "8 64" "64 40" "64 64"; do set -- $V
    timeout -k 10 200 python bench.py --total-envs $1 --substeps $2 --steps 256 --warmup 64 --no-cpu-baseline > $O/e$1_s$2.json 2> $O/err || { tail -20 $O/err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'ms/step %.4f' % d['ms_per_step'], d['check']['ok'])" $O/e$1_s$2.json
  done
done
