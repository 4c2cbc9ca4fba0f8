# Round 5: k_rollout at training-sized batches (8192 / 32768 / 131072 envs, 64x64) + 256x256 4096-env chunk check.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05t}
mkdir -p $O
export TMPDIR=/tmp
for E in 8192 32768 131072 8192; do
timeout -k 10 300 python bench.py --envs $E --no-cpu-baseline > $O/e$E.json 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/e$E.json')); r=d['roofline']; print('E=$E %.4e frac %.4f ms/step %.4f kernel_ms %.3f spl %s check %s' % (d['value'], r['frac'], d['ms_per_step'], r.get('kernel_ms', -1), d['config'].get('steps_per_launch'), d.get('check', {}).get('ok')))"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof8192 -o r -- python3 $GRAFT_REPO_ROOT/bench.py --envs 8192 --no-cpu-baseline --steps 20 --warmup 4 > $GRAFT_REPO_ROOT/$O/prof8192.json 2> $GRAFT_REPO_ROOT/$O/prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT && python3 -c "
import csv, collections
rows=[r for r in csv.DictReader(open('$O/prof8192/r_kernel_trace.csv')) if 'k_rollout' in r['Kernel_Name']]
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows]
print('k_rollout launches', len(d), 'us: mean %.1f min %.1f max %.1f' % (sum(d)/len(d), min(d), max(d)))
"
timeout -k 10 300 python bench.py --map 256 --agents 4096 --envs 4096 --substeps 20 --steps 60 --warmup 10 --check-envs 2 --no-cpu-baseline > $O/e256_4096.json 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/e256_4096.json')); r=d['roofline']; print('256 E=4096 %.4e frac %.4f ms/step %.4f check %s' % (d['value'], r['frac'], d['ms_per_step'], d.get('check', {}).get('ok')))"
