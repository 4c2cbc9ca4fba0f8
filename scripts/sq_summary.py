"""SQ wave-state counters of the last N k_rollout dispatches of one rocprofv3 --pmc pass -> JSON.

    python scripts/sq_summary.py <run_counter_collection.csv> [N] [note] [kernel substring, default k_rollout]
SQ_* are quad-cycles summed over waves (and SIMDs); GRBM_GUI_ACTIVE is summed over the 8 XCDs."""
import collections
import csv
import json
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
kname = sys.argv[4] if len(sys.argv) > 4 else "k_rollout"
by = collections.defaultdict(lambda: collections.defaultdict(float))
order = []
for r in csv.DictReader(open(path)):
    if kname not in r["Kernel_Name"]:
        continue
    d = r["Dispatch_Id"]
    if d not in by:
        order.append(d)
    by[d][r["Counter_Name"]] += float(r["Counter_Value"])
last = order[-n:]
avg = {c: sum(by[d][c] for d in last) / len(last) for c in by[last[0]]}
wc = avg["SQ_WAVE_CYCLES"]
cyc = avg["GRBM_GUI_ACTIVE"] / 8.0
avg["derived"] = {
    "wait_any_frac": avg["SQ_WAIT_ANY"] / wc,
    "wait_inst_any_frac": avg["SQ_WAIT_INST_ANY"] / wc,
    "active_inst_any_frac": avg["SQ_ACTIVE_INST_ANY"] / wc,
    "valu_busy_per_simd": avg["SQ_ACTIVE_INST_VALU"] * 4 / (cyc * 256 * 4),
    "waves_resident_mean": wc * 4 / cyc,
}
avg["note"] = (sys.argv[3] if len(sys.argv) > 3 else "") + "; mean of the last %d %s dispatches" % (len(last), kname)
print(json.dumps(avg, indent=1))
