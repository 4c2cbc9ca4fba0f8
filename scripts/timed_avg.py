"""Average k_rollout duration over the last N launches (the timed region) of a rocprofv3 kernel trace.

    python scripts/timed_avg.py <run_kernel_trace.csv> <N>"""
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'k_rollout' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
n = int(sys.argv[2])
d = [int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in rows]
print(f"k_rollout launches: {len(d)}; all avg {sum(d)/len(d)/1e6:.4f} ms; last {n} (timed region) avg {sum(d[-n:])/n/1e6:.4f} ms; first {len(d)-n} avg {sum(d[:-n])/(len(d)-n)/1e6:.4f} ms")
