# Round 6: the 32768-env split line's self-check failure (engine 1, env 16383, group 1 ids) was the checker's: its
# getters ran on the engine's stream, torch's index_select on the current one (tests/rollout_check.py, fixed).  Rerun
# with 16 checked envs, and the split lines at 4096 / 8192 / 12288 / 16384 envs, same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r06g}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --total-envs 32768 --split 2 --steps 256 --warmup 64 --no-cpu-baseline --no-ceiling --check-envs 16 > $O/b32768_2.json 2> $O/err_1 || { tail -5 $O/err_1; exit 1; }
python3 -c "import json; d=json.load(open('$O/b32768_2.json')); c=d['check']; print('32768 split 2', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], c['ok'], c['sample_rank0'], c['mismatches'])"
for r in 1 2; do
for E in 4096 8192 12288 16384; do
for H in 1 2; do
timeout -k 10 200 python bench.py --total-envs $E --split $H --steps 256 --warmup 64 --no-cpu-baseline --check-envs 4 > $O/b_${E}_${H}_$r.json 2> $O/err || { tail -20 $O/err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_${E}_${H}_$r.json')); r=d['roofline']; print('$E envs split $H', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'frac %.4f' % r['frac'], 'frac_measured %.4f' % r['frac_measured'], 'S', d['config']['steps_per_launch'], 'check', d['check']['ok'])"
done
done
done
