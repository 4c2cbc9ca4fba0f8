# A/B of two library builds on one box, interleaved: scripts/gpu_ab.sh VARIANT [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
V=$1; shift
for r in 1 2 3; do for lib in libmagent libmagent_$V; do
MAGENT_LIB=$L/$lib.so timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_${lib}_$r.json 2> gpurun_out/ab.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/ab_${lib}_$r.json')); print('$lib', $r, '%.4e' % d['value'], '%.4f' % d['ms_per_step'])"
done; done
