# Round 4: small-batch k_rollout -- the 8192-env timeline with restart attribution, and steps per launch at
# 8192 / 32768 envs (S = 5 / 10 / 20), the queue as committed.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04e}
mkdir -p $O
export TMPDIR=/tmp
L=mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so
MAGENT_LIB=$L timeout -k 10 200 python scripts/timeline_rollout.py --envs 8192 --substeps 20 > $O/tl_8192.txt 2>&1 || { tail -20 $O/tl_8192.txt; exit 1; }
cat $O/tl_8192.txt
for rep in 1 2; do for E in 8192 32768; do for S in 5 10 20; do
  timeout -k 10 300 python bench.py --envs $E --substeps $S --steps 60 --warmup 10 --no-cpu-baseline --check-envs 2 > $O/e${E}_s$S.json 2> $O/err || { tail -20 $O/err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], '%.4e' % d['value'], '%.4f' % d['roofline']['frac'], '%.4f' % d['ms_per_step'], d['check']['ok'])" $O/e${E}_s$S.json
done; done; done
