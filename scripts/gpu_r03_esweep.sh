# Round 3: 64x64 envs per GPU x steps per launch on the final tree, interleaved on one box (self-checked lines).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/esweep}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in "49152 4" "65536 4" "98304 4" "49152 8" "65536 8"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --envs $1 --substeps $2 --steps 40 --warmup 8 --no-cpu-baseline > $O/e$1_s$2_$r.json 2> $O/e$1_s$2_$r.err || { tail -20 $O/e$1_s$2_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e$1_s$2_$r.json')); print('envs $1 sub $2', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
  done
done
