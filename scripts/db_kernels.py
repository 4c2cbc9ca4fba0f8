"""Kernel dispatches of a rocprofv3 results database (rocpd sqlite, the default output): per kernel name the
count, total / mean / last durations (ms), optionally only the last N dispatches of each.

    python scripts/db_kernels.py <results.db> [--last N] [--match substring]"""
import argparse
import collections
import json
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--last", type=int, default=0)
ap.add_argument("--match", default="")
a = ap.parse_args()
cur = sqlite3.connect(a.db).cursor()
by = collections.defaultdict(list)
for name, start, dur in cur.execute("select name, start, duration from kernels order by start"):
    if a.match in name:
        by[name].append(dur / 1e6)
out = {}
for name, d in by.items():
    sel = d[-a.last:] if a.last else d
    out[name.split("(")[0][:90]] = {"count": len(d), "used": len(sel), "total_ms": sum(sel),
                                    "mean_ms": sum(sel) / len(sel), "last_ms": d[-1]}
print(json.dumps(out, indent=1))
