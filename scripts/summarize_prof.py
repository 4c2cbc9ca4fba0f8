"""Summarize rocprofv3 outputs of the bench for profiles/: kernel stats + per-launch HBM bytes.

    python scripts/summarize_prof.py <prof_dir> <pmc_fetch_dir> <pmc_write_dir> <envs> <out_json>
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE reads 1/2 of a wide
coalesced stream (MI355X_MICROARCH.md, HBM) so it is doubled; WRITE_SIZE is exact for 16-B stores.
Only k_rollout dispatches of the timed part are used (the last `steps` launches)."""
import csv
import json
import sys


def per_launch(path, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if "k_rollout" in r["Kernel_Name"] and r["Counter_Name"] == counter]
    tail = vals[-20:]
    return sum(tail) / len(tail), len(vals)


prof, fetch, write, envs, out = sys.argv[1:6]
stats = list(csv.DictReader(open(prof + "/run_kernel_stats.csv")))
trace = [r for r in csv.DictReader(open(prof + "/run_kernel_trace.csv")) if "k_rollout" in r["Kernel_Name"]]
dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace]
f_kib, nf = per_launch(fetch + "/run_counter_collection.csv", "FETCH_SIZE")
w_kib, nw = per_launch(write + "/run_counter_collection.csv", "WRITE_SIZE")
res = {
    "envs": int(envs),
    "kernel_stats": [{k: r[k] for k in ("Name", "Calls", "AverageNs", "MinNs", "MaxNs", "Percentage")} for r in stats],
    "k_rollout_timed_avg_ns": sum(dur[-60:]) / len(dur[-60:]),
    "k_rollout_all_avg_ns": sum(dur) / len(dur),
    "fetch_size_kib_per_launch_raw": f_kib,
    "write_size_kib_per_launch": w_kib,
    "hbm_read_bytes_per_launch": 2 * f_kib * 1024,
    "hbm_write_bytes_per_launch": w_kib * 1024,
    "hbm_bytes_per_launch": (2 * f_kib + w_kib) * 1024,
    "note": "FETCH_SIZE doubled (gfx950 tallies 128-B requests at 64 B); last 20 k_rollout dispatches of each PMC pass",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
