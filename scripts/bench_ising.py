"""Ising tabular MF-Q throughput (configs[0]: 20x20 lattice, tau = 0.8, lr 0.1, act_rate 1.0):
spin-steps/s of k_ising_mfq over R independent replicas (Philox draws on device; one launch runs
each replica's whole episode incl. the early stop of main_MFQ_Ising.py), next to the vectorised
numpy restatement of the script (oracle/ising_oracle.py, one host thread) on the same box.

    python scripts/bench_ising.py [--replicas R] [--steps T]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

ap = argparse.ArgumentParser()
ap.add_argument("--replicas", type=int, default=4096)
ap.add_argument("--steps", type=int, default=2000)
ap.add_argument("--cpu-seconds", type=float, default=10.0)
a = ap.parse_args()

import torch  # noqa: E402
from mfrl_amd.ising import run_mfq  # noqa: E402
import ising_oracle  # noqa: E402

torch.cuda.set_device(0)
run_mfq(400, 0.8, 50, mode="philox", replicas=64, seed=1)              # warm-up
torch.cuda.synchronize()
t0 = time.perf_counter()
res = run_mfq(400, 0.8, a.steps, mode="philox", replicas=a.replicas, seed=7)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
done = int(res["steps"].sum())
gpu = done * 400 / dt
# CPU: the numpy restatement of the reference loop, episodes of the same length
t0, cpu_steps = time.perf_counter(), 0
while time.perf_counter() - t0 < a.cpu_seconds:
    r = ising_oracle.mfq(400, 0.8, min(a.steps, 500), seed=13 + cpu_steps)
    cpu_steps += r["steps"]
cdt = time.perf_counter() - t0
line = {"metric": "spin-steps/sec Ising 20x20 tabular MF-Q", "value": gpu, "unit": "spin-steps/s",
        "replicas": a.replicas, "steps_cap": a.steps, "steps_run": done, "seconds": dt,
        "bytes_per_spin_step": 41, "achieved_GBs": gpu * 41 / 1e9,
        "cpu_baseline": {"value": cpu_steps * 400 / cdt, "unit": "spin-steps/s", "cores": 1, "kind": "port",
                         "sample": "%d steps of 500-step episodes, oracle/ising_oracle.py (numpy)" % cpu_steps}}
print(json.dumps(line))
