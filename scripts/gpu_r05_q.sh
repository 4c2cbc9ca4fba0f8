# Round 5: 256x256 steps-per-launch and batch anomalies: 2048 envs at S = 20 / 32 / 40 / 64 and
# 3072 envs at S = 20, kernel traces for the launch durations.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05q}
mkdir -p $O
export TMPDIR=/tmp
for C in "2048 20" "2048 40" "2048 32" "2048 64" "3072 20" "2048 20"; do
set -- $C; E=$1; S=$2
timeout -k 10 300 python bench.py --map 256 --agents 4096 --envs $E --substeps $S --steps 96 --warmup 16 --check-envs 2 --no-cpu-baseline > $O/e${E}_s$S.json 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/e${E}_s$S.json')); r=d['roofline']; print('E=$E S=$S %.4e frac %.4f ms/step %.4f kernel_ms %.3f check %s' % (d['value'], r['frac'], d['ms_per_step'], r.get('kernel_ms', -1), d.get('check', {}).get('ok')))"
done
