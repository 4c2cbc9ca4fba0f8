# Round 5: the few-env snapshot from a per-launch context in LDS with one flat 16-B copy: parity, stamps, 8-env bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05ad}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "few or small_e or two_engines" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
MAGENT_LIB=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 300 python scripts/stamps_few.py --envs 8 --sub 20 --launches 20 --snap > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
grep -v amdgpu.ids $O/stamps.txt
for E in 8 64 8; do
timeout -k 10 300 python bench.py --total-envs $E --steps 256 --warmup 32 --no-cpu-baseline > $O/b$E.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b$E.json')); print('E=$E %.4e ms/step %.4f check %s' % (d['value'], d['ms_per_step'], d.get('check', {}).get('ok')))"
done
