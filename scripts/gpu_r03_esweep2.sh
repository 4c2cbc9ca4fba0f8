# Round 3: the larger 64x64 batches -- envs per GPU x steps per launch, interleaved on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/esweep2
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in "49152 4" "98304 4" "98304 8" "131072 4" "131072 8" "65536 8"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --envs $1 --substeps $2 --steps 40 --warmup 8 --no-cpu-baseline > $O/e$1_s$2_$r.json 2> $O/e$1_s$2_$r.err || { tail -20 $O/e$1_s$2_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/e$1_s$2_$r.json')); print('envs $1 sub $2', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'], 'ms/step %.3f' % d['ms_per_step'])"
  done
done
