"""Summarize rocprofv3 outputs of the bench for profiles/: kernel stats + per-launch HBM bytes.

    python scripts/summarize_prof.py <prof_dir> <pmc_fetch_dir> <pmc_write_dir> <envs> <out_json>
                                     [substeps timed_launches pmc_launches [map bench_json]]
bench_json (the profiled bench line): adds agent-steps per launch and HBM bytes per agent-step.
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE reads 1/2 of a wide
coalesced stream (MI355X_MICROARCH.md, HBM) so it is doubled; WRITE_SIZE is exact for 16-B stores.
Only k_rollout dispatches of the timed part are used (the last `timed_launches` launches of the trace,
the last `pmc_launches` of each PMC pass); one launch runs `substeps` steps of every env."""
import csv
import hashlib
import json
import os
import sys

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "mean-field-multi-agent-reinforcement-learning_amd", "build", "libmagent.so")


def per_launch(path, counter, n):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if "k_rollout" in r["Kernel_Name"] and r["Counter_Name"] == counter]
    tail = vals[-n:]
    return sum(tail) / len(tail), len(vals)


prof, fetch, write, envs, out = sys.argv[1:6]
sub, timed, npmc = (int(x) for x in (sys.argv[6:9] if len(sys.argv) > 8 else (1, 60, 20)))
stats = list(csv.DictReader(open(prof + "/run_kernel_stats.csv")))
trace = [r for r in csv.DictReader(open(prof + "/run_kernel_trace.csv")) if "k_rollout" in r["Kernel_Name"]]
dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace]
f_kib, nf = per_launch(fetch + "/run_counter_collection.csv", "FETCH_SIZE", npmc)
w_kib, nw = per_launch(write + "/run_counter_collection.csv", "WRITE_SIZE", npmc)
res = {
    "envs": int(envs),
    # the library build the counters were collected on (bench.py attaches them only to lines of the same build)
    "lib_sha16": hashlib.sha256(open(LIB, "rb").read()).hexdigest()[:16],
    "substeps": sub,
    "kernel_stats": [{k: r[k] for k in ("Name", "Calls", "AverageNs", "MinNs", "MaxNs", "Percentage")} for r in stats],
    "k_rollout_timed_avg_ns": sum(dur[-timed:]) / len(dur[-timed:]),
    "k_rollout_timed_launches": timed,
    "k_rollout_all_avg_ns": sum(dur) / len(dur),
    "fetch_size_kib_per_launch_raw": f_kib,
    "write_size_kib_per_launch": w_kib,
    "hbm_read_bytes_per_launch": 2 * f_kib * 1024,
    "hbm_write_bytes_per_launch": w_kib * 1024,
    "hbm_bytes_per_launch": (2 * f_kib + w_kib) * 1024,
    "note": "FETCH_SIZE doubled (gfx950 tallies 128-B requests at 64 B); last %d k_rollout dispatches of each PMC "
            "pass; %d step(s) of every env per launch" % (npmc, sub),
}
if len(sys.argv) > 10:
    line = json.load(open(sys.argv[10]))
    units = line["roofline"]["units_per_launch"]
    res.update({"map": int(sys.argv[9]), "agent_steps_per_launch": units,
                "hbm_bytes_per_agent_step": res["hbm_bytes_per_launch"] / units,
                "algorithmic_bytes_per_agent_step": line["roofline"]["bytes_per_unit"],
                "ratio": res["hbm_bytes_per_launch"] / units / line["roofline"]["bytes_per_unit"],
                "bench_kernel_ms": line["roofline"]["kernel_ms"], "bench_value": line["value"]})
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
