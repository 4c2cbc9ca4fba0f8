# Round 3: 256x256 envs per GPU x steps per k_rollout_bigq launch after the slot renumbering, interleaved on one
# box, every line self-checked on the oracle.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sw256
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in "1024 16" "2048 16" "2048 32" "3072 32" "1024 32"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --map 256 --agents 4096 --envs $1 --substeps $2 --steps 64 --warmup 16 --no-cpu-baseline > $O/e$1_s$2_$r.json 2> $O/e$1_s$2_$r.err || { tail -20 $O/e$1_s$2_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e$1_s$2_$r.json')); print('envs $1 sub $2', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
  done
done
