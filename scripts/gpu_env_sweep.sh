# Throughput against the number of envs per GPU (same binary, one box): scripts/gpu_env_sweep.sh "4096 8192 ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do for E in $1; do
timeout -k 10 300 python bench.py --no-cpu-baseline --envs $E > gpurun_out/envs_${E}_$r.json 2> gpurun_out/envs.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/envs_${E}_$r.json')); print($E, $r, '%.4e' % d['value'], 'ms %.4f' % d['ms_per_step'])"
done; done
