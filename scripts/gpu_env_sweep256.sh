# 256x256 / 4096 agents throughput against envs per GPU: scripts/gpu_env_sweep256.sh "1024 1536 ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do for E in $1; do
timeout -k 10 300 python bench.py --no-cpu-baseline --map 256 --agents 4096 --envs $E > gpurun_out/envs256_${E}_$r.json 2> gpurun_out/envs.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/envs256_${E}_$r.json')); print($E, $r, '%.4e' % d['value'], 'ms %.4f' % d['ms_per_step'])"
done; done
