# Round 4: 2-rank gloo rehearsals on one card after routing shared-card ranks off the queue kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04v}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --total-envs 16 --steps 256 --warmup 64 --no-cpu-baseline > $O/bench_2rank_16envs.json 2> $O/e1.err || { tail -20 $O/e1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2rank_16envs.json')); print('2 ranks x 8 envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], d['config']['workload'], d['config']['parallelism'], 'check', d['check']['ok'])"
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --map 256 --agents 4096 --envs 64 --steps 8 --warmup 2 --no-cpu-baseline > $O/bench_2rank_256.json 2> $O/e2.err || { tail -20 $O/e2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2rank_256.json')); print('2 ranks 256x256', '%.4e' % d['value'], d['config']['workload'], 'check', d['check']['ok'])"
timeout -k 10 200 python scripts/bench_dropin.py --map 40 --agents 128 --seconds 4 --calls > $O/dropin_40.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/dropin_40.json')); print('drop-in 40x40 vs ref', '%.3f' % d['hip_vs_ref'])"
