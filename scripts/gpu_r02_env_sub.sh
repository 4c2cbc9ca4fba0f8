# k_rollout (64x64): envs per GPU x steps per launch, interleaved, two runs each (no CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02e
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in "24576 4" "32768 4" "49152 4" "24576 6" "32768 8"; do
    set -- $cfg
    timeout -k 10 200 python bench.py --envs $1 --substeps $2 --steps 48 --warmup 8 --no-cpu-baseline > $O/e$1_s$2_$r.json 2> $O/e$1_s$2_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/e$1_s$2_$r.json')); print('envs $1 sub $2', '%.4g'%d['value'], '%.3f'%d['roofline']['frac'])"
  done
done
