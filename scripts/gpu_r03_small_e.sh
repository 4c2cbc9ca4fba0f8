# configs[3] shape on one GPU (8 and 64 envs): k_rollout (one workgroup per env) vs the queue kernel
# k_rollout_bigq (MFX_SMALL_E) with 16 / 32 / 64-agent items; every line self-checked on the oracle.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03e
mkdir -p $O
for E in 8 64; do
  timeout -k 10 120 python bench.py --total-envs $E --steps 200 --warmup 20 --no-cpu-baseline > $O/k_rollout_$E.json 2> $O/err || { tail -5 $O/err; exit 1; }
  python -c "import json;d=json.load(open('$O/k_rollout_$E.json'));print('E=$E k_rollout', d['value'], d['ms_per_step'], d['check']['ok'])"
  for R in 16 32 64; do
    for S in 4 16; do
      MFX_SMALL_E=64 MFX_BIGQ_ROWS=$R timeout -k 10 120 python bench.py --total-envs $E --substeps $S --steps 192 --warmup 16 --no-cpu-baseline > $O/bigq_${E}_${R}_${S}.json 2> $O/err || { tail -5 $O/err; exit 1; }
      python -c "import json;d=json.load(open('$O/bigq_${E}_${R}_${S}.json'));print('E=$E bigq R=$R S=$S', d['config']['workload'][-40:], d['value'], d['ms_per_step'], d['check']['ok'])"
    done
  done
done
