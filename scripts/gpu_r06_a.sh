# Round 6 start: same-box baseline of the lines the round works on (64x64 default, 8192 envs, MFAC loop).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r06a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('64x64', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'check', d['check']['ok'])"
for E in 8192 32768; do
timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/bench_${E}envs.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_${E}envs.json')); print('$E envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'frac %.4f' % d['roofline']['frac'], 'S', d['config']['steps_per_launch'], 'check', d['check']['ok'])"
done
timeout -k 10 300 python bench.py --policy mfac --no-cpu-baseline > $O/bench_mfac.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_mfac.json')); print('mfac', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'fwd ms %.3f' % d['roofline']['kernel_ms'], 'ms/step %.3f' % d['ms_per_step'])"
