# Round 6: after the A/B knob removal (queue tiers fixed, pipelined few-env overlap fixed, the one-wave QNet conv and
# the batched row movers gone): the whole GPU suite, the bench lines at every shape the round touches.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r06e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --durations=15 --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('64x64', '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'measured_peak %.0f' % r['measured_peak'], 'frac_measured %.4f' % r['frac_measured'], 'check', d['check']['ok'])"
for E in 8 64 8192 32768; do
timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline > $O/bench_${E}envs.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_${E}envs.json')); r=d['roofline']; print('$E envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'frac %.4f' % r['frac'], 'frac_measured', r['frac_measured'], 'S', d['config']['steps_per_launch'], 'check', d['check']['ok'])"
done
timeout -k 10 400 python bench.py --map 256 --agents 4096 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench256.json 2> $O/bench256.err || { tail -20 $O/bench256.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench256.json')); r=d['roofline']; print('256x256', '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'frac_measured %.4f' % r['frac_measured'], 'check', d['check']['ok'])"
MFX_ROWS_PIPE=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_replay_gpu.py tests/test_algo_gpu.py > $O/tests_x4.log 2>&1 || { tail -30 $O/tests_x4.log; exit 1; }
tail -1 $O/tests_x4.log
L=mean-field-multi-agent-reinforcement-learning_amd/build
for r in 1 2; do
for V in "1 libmagent" "2 libmagent" "2 libmagent_rows2" "2 libmagent_rows8"; do
set -- $V
MFX_ROWS_PIPE=$1 MAGENT_LIB=$L/$2.so timeout -k 10 200 python scripts/bench_replay.py --cpu-seconds 0.5 > $O/replay_$1_$2_$r.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/replay_$1_$2_$r.json')); print('replay pipe=$1 $2', '%.4e rows/s' % d['value'], 'frac %.4f' % d['roofline']['frac'])"
done
done
timeout -k 10 600 python scripts/exp_split_rollout.py --envs 8192 --splits 1 2 4 --substeps 0 2 20 > $O/split8192.jsonl 2> $O/err || { tail -20 $O/err; exit 1; }
cat $O/split8192.jsonl
