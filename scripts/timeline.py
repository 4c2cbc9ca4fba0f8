"""Kernel-trace timeline summary (rocprofv3 --kernel-trace csv): busy fraction and overlap in the last window.

    python scripts/timeline.py <prof_dir> [last_n_kernels]"""
import csv
import sys
from collections import defaultdict

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 120
rows = [r for r in csv.DictReader(open(d + "/run_kernel_trace.csv"))]
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows)
ks = [k for k in ks if "rocclr" not in k[2]][-n:]
t0, t1 = ks[0][0], max(k[1] for k in ks)
ev = sorted([(a, 1) for a, _, _ in ks] + [(b, -1) for _, b, _ in ks])
busy, cur, last, acc = 0, 0, t0, defaultdict(int)
for t, dlt in ev:
    if cur > 0:
        busy += t - last
    acc[cur] += t - last
    cur += dlt
    last = t
dur = defaultdict(list)
for a, b, k in ks:
    dur[k].append(b - a)
print("window %.1f us over %d kernels: busy %.1f%%" % ((t1 - t0) / 1e3, len(ks), 100.0 * busy / (t1 - t0)))
print("time at concurrency level:", {c: "%.1f%%" % (100.0 * v / (t1 - t0)) for c, v in sorted(acc.items())})
for k, v in dur.items():
    print("  %-40s n=%d avg %.1f us" % (k[-40:], len(v), sum(v) / len(v) / 1e3))
