# Round 4: instruction-cache counters of the few-env rollout (configs[3] shape, 8 envs) -- pipelined vs queue step.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04m}
mkdir -p $O
export TMPDIR=/tmp
for P in 1 0; do
  MFX_FEW_PIPE=$P timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
      -d $O/ic_p$P -o ic --output-format csv -- python3 bench.py --total-envs 8 --steps 40 --warmup 5 --no-cpu-baseline --check-envs 0 > $O/ic_p$P.log 2>&1 || { tail -20 $O/ic_p$P.log; exit 1; }
  python3 - $O/ic_p$P <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = {}
for r in csv.DictReader(open(f)):
    if "k_rollout_bigq" in r["Kernel_Name"]:
        d = acc.setdefault(r["Dispatch_Id"], {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
vals = list(acc.values())
print(sys.argv[1], "dispatches", len(vals), "last 3:", vals[-3:])
PY
done
