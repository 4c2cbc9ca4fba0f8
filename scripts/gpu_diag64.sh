set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
for r in 1 2; do for lib in libmagent libmagent_obsonly libmagent_noobs; do
MAGENT_LIB=$L/$lib.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 --warmup 5 > gpurun_out/diag_${lib}_$r.json 2> gpurun_out/diag.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/diag_${lib}_$r.json')); print('$lib', $r, '%.4e' % d['value'], 'ms %.4f' % d['ms_per_step'], 'achieved %.0f GB/s' % d['roofline']['achieved'])"
done; done
