"""Durations of the kernels whose name contains a substring, from a rocprofv3 --kernel-trace csv.

    python scripts/kernel_durations.py <run_kernel_trace.csv> <substring> [last_n]"""
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
if len(sys.argv) > 3:
    rows = rows[-int(sys.argv[3]):]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
print(json.dumps({"kernel": sys.argv[2], "launches": len(d), "ms": d[-8:], "avg_ms": sum(d) / max(1, len(d)),
                  "max_ms": max(d) if d else None, "grid": rows[-1].get("Grid_Size") if rows else None,
                  "workgroup": rows[-1].get("Workgroup_Size") if rows else None}))
