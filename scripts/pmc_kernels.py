"""Per-kernel average of one rocprofv3 counter over the last N dispatches of each kernel.

    python scripts/pmc_kernels.py <counter_collection.csv> <counter> [N]
FETCH_SIZE is printed as read (KiB; gfx950 tallies wide requests at half size, so HBM read bytes are
2x this, MI355X_MICROARCH.md) and WRITE_SIZE as read (KiB)."""
import csv
import json
import sys

path, counter = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
per = {}
for r in csv.DictReader(open(path)):
    if r["Counter_Name"] != counter:
        continue
    name = r["Kernel_Name"].split("(")[0]
    per.setdefault(name, []).append(float(r["Counter_Value"]))
out = {k: {"dispatches": len(v), "avg_kib_last": sum(v[-n:]) / len(v[-n:])} for k, v in per.items()}
print(json.dumps({"counter": counter, "last": n, "kernels": out}, indent=1))
