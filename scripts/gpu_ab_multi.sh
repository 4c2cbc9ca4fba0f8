# Interleaved A/B of several library builds on one box: scripts/gpu_ab_multi.sh "V1 V2 ..." [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
VS=$1; shift
for r in 1 2; do for v in base $VS; do
lib=libmagent; [ $v != base ] && lib=libmagent_$v
MAGENT_LIB=$L/$lib.so timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/abm_${v}_$r.json 2> gpurun_out/abm.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/abm_${v}_$r.json')); print('$v', $r, '%.4e' % d['value'], 'ms %.4f' % d['ms_per_step'])"
done; done
