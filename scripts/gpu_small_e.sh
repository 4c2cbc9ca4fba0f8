set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
for E in 8 64; do for lib in libmagent libmagent_head; do
MAGENT_LIB=$L/$lib.so timeout -k 10 300 python bench.py --no-cpu-baseline --envs $E --steps 200 --warmup 10 > gpurun_out/se_${lib}_$E.json 2> gpurun_out/se.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/se_${lib}_$E.json')); print('$lib', $E, '%.4e' % d['value'], '%.4f' % d['ms_per_step'])"
done; done
