# Round 5: is the few-env stepper instruction-fetch bound?  -Os build (A/B only) vs the product build, 8 envs, plus the
# instruction-cache counters of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05af}
mkdir -p $O
export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
for V in "" _os "" _os; do
MAGENT_LIB=$B/libmagent$V.so timeout -k 10 300 python bench.py --total-envs 8 --steps 256 --warmup 32 --no-cpu-baseline > $O/b$V.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b$V.json')); print('lib$V %.4e ms/step %.4f check %s' % (d['value'], d['ms_per_step'], d.get('check', {}).get('ok')))"
done
for V in "" _os; do
cd /tmp && MAGENT_LIB=$B/libmagent$V.so timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d $GRAFT_REPO_ROOT/$O/ic$V -o ic --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --total-envs 8 --steps 40 --warmup 5 --no-cpu-baseline --check-envs 0 > $GRAFT_REPO_ROOT/$O/ic$V.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/ic$V.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 - $O/ic$V <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = {}
for r in csv.DictReader(open(f)):
    if "k_rollout_bigq" in r["Kernel_Name"]:
        d = acc.setdefault(r["Dispatch_Id"], {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
vals = list(acc.values())
print(sys.argv[1], "dispatches", len(vals), "last 2:", vals[-2:])
PY
done
