# Interleaved bench runs over values of one environment knob: scripts/gpu_env_knob.sh VAR "v1 v2 ..." [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VAR=$1; VALS=$2; shift 2
for r in 1 2; do for x in $VALS; do
env $VAR=$x timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/knob_${x}_$r.json 2> gpurun_out/knob.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/knob_${x}_$r.json')); print('$VAR=$x', $r, '%.4e' % d['value'], 'ms %.4f' % d['ms_per_step'])"
done; done
