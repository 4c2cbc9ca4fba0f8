#!/bin/bash
# Round 6 final refresh, part 1: the whole GPU suite, smoke, and the bench lines on the committed build (default with
# the CPU baseline and the measured ceiling, 256x256, configs[3] shapes, 8192 envs, the 2-rank gloo rehearsals, the
# learned policies, Ising, the drop-in, the replay mover, the generic configs).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r06_final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --durations=15 --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('64x64', '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'measured', r.get('measured_peak'), 'frac_measured', r.get('frac_measured'), 'traffic', r.get('traffic'), 'check', d['check']['ok'], 'cpu', '%.3e' % d['cpu_baseline']['value'])"
timeout -k 10 400 python bench.py --map 256 --agents 4096 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench256.json 2> $O/bench256.err || { tail -20 $O/bench256.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench256.json')); r=d['roofline']; print('256x256', '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'frac_measured', r.get('frac_measured'), 'check', d['check']['ok'])"
for E in 8 64; do
timeout -k 10 200 python bench.py --total-envs $E --steps 256 --warmup 64 --no-cpu-baseline --no-ceiling > $O/bench_${E}envs.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_${E}envs.json')); print('$E envs', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'check', d['check']['ok'])"
done
timeout -k 10 200 python bench.py --envs 8192 --no-cpu-baseline > $O/bench_8192envs.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_8192envs.json')); r=d['roofline']; print('8192 envs', '%.4e' % d['value'], 'frac %.4f' % r['frac'], 'frac_measured', r.get('frac_measured'), 'check', d['check']['ok'])"
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --envs 2048 --steps 20 --warmup 3 --no-cpu-baseline --no-ceiling > $O/bench_2rank.json 2> $O/bench_2rank.err || { tail -20 $O/bench_2rank.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_2rank.json')); print('2 ranks', '%.4e' % d['value'], d['config']['parallelism'], d['check']['ok'])"
for P in qnet mfac; do
timeout -k 10 300 python bench.py --policy $P --no-cpu-baseline --no-ceiling > $O/bench_$P.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_$P.json')); print('$P', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'])"
done
timeout -k 10 400 python scripts/bench_ising.py --mode reference > $O/ising_reference.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/ising_reference.json')); print('ising reference', d['replicas'], '%.4e' % d['value'], d['check'])"
timeout -k 10 200 python scripts/bench_dropin.py --map 40 --agents 128 --seconds 4 --calls > $O/dropin_40.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/dropin_40.json')); print('drop-in 40x40 vs ref', '%.3f' % d['hip_vs_ref'])"
timeout -k 10 120 python -u scripts/bench_replay.py --cpu-seconds 2 > $O/replay.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/replay.json')); print('replay', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'])"
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent.so
for cfg in "double_attack 24 40,60" "forest 32 60,50"; do
  set -- $cfg
  timeout -k 10 120 python -u scripts/bench_generic.py --lib $L --config $1 --map $2 --counts $3 >> $O/generic.jsonl 2> $O/err || { tail -20 $O/err; exit 1; }
  tail -1 $O/generic.jsonl | cut -c1-200
done
