"""Ising tabular MF-Q throughput (configs[0]: 20x20 lattice, tau = 0.8, lr 0.1, act_rate 1.0): spin-steps/s of
k_ising_mfq over R independent replicas, one launch running each replica's whole episode incl. the early stop of
main_MFQ_Ising.py -- next to two CPU baselines on the same box, one core each: the vectorised numpy restatement
(oracle/ising_oracle.py mfq) and the reference's per-agent loop restated as the script runs it (mfq_loop).

    python scripts/bench_ising.py [--mode philox|reference] [--replicas R] [--steps T]

mode philox: the uniforms are drawn on the device (perf mode, statistically checked); reference: every replica
consumes its own numpy RandomState stream generated on the host (bit-exact to main_MFQ_Ising.py: uploaded as
8 B per spin-step, the kernel's only HBM read).  `value` is the host clock around mfx_ising_mfq_run (the
upload of the streams, the launch, the read-back of Q / order / n_up); the kernel alone is read from a rocprofv3
kernel trace of the same command (scripts/kernel_durations.py)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

ap = argparse.ArgumentParser()
ap.add_argument("--mode", choices=("philox", "reference"), default="philox")
ap.add_argument("--replicas", type=int, default=None, help="default 16384 (philox) / 256 (reference)")
ap.add_argument("--steps", type=int, default=2000)
ap.add_argument("--cpu-seconds", type=float, default=10.0)
ap.add_argument("--no-cpu", action="store_true")
a = ap.parse_args()
R = a.replicas or (16384 if a.mode == "philox" else 256)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import ising_oracle  # noqa: E402
from mfrl_amd.ising import IsingLattice, reference_stream  # noqa: E402

N = 400
torch.cuda.set_device(0)
lat = IsingLattice(N, R)
if a.mode == "reference":
    t0 = time.perf_counter()
    streams = [reference_stream(13 + r, N, a.steps) for r in range(R)]
    gen_s = time.perf_counter() - t0
    spins0 = np.stack([s[0] for s in streams])
    u = np.stack([s[1] for s in streams])
    del streams
else:
    spins0 = np.random.RandomState(7).randint(0, 2, size=(R, N))
    u, gen_s = None, 0.0
warm = IsingLattice(N, 64)                                              # warm-up launch (code objects, buffers)
warm.set_spins(spins0[:64])
warm.run_mfq(50, 0.8, u=u[:64, :50] if u is not None else None, seed=1)
lat.set_spins(spins0)
torch.cuda.synchronize()
t0 = time.perf_counter()
res = lat.run_mfq(a.steps, 0.8, u=u, seed=7)
dt = time.perf_counter() - t0
done = int(res["steps"].sum())
line = {"metric": "spin-steps/sec Ising 20x20 tabular MF-Q (%s mode)" % a.mode,
        "value": done * N / dt, "unit": "spin-steps/s", "mode": a.mode, "replicas": R, "steps_cap": a.steps,
        "steps_run": done, "seconds_call": dt,
        "call_is": "mfx_ising_mfq_run: %s the launch and the read-back of Q / order / n_up"
                   % ("upload of the host streams (8 B per spin-step), " if u is not None else ""),
        "host_stream_generation_s": gen_s,
        "steps_mean": float(res["steps"].mean())}
if a.mode == "reference":                                               # the replicas' results vs the numpy oracle
    bad = 0
    for r in range(0, R, max(1, R // 4)):
        ref = ising_oracle.mfq(N, 0.8, a.steps, seed=13 + r)
        bad += int(ref["steps"] != int(res["steps"][r]) or ref["q"].tobytes() != res["q"][r].tobytes())
    line["check"] = {"replicas_compared": len(range(0, R, max(1, R // 4))), "mismatches": bad,
                     "what": "Q table and episode length bit for bit against oracle/ising_oracle.py"}
if not a.no_cpu:
    cpu = {}
    for name, fn, cap in (("numpy_port", ising_oracle.mfq, 500), ("per_agent_loop", ising_oracle.mfq_loop, 40)):
        t0, n_steps, k = time.perf_counter(), 0, 0
        while time.perf_counter() - t0 < a.cpu_seconds / 2:
            r = fn(N, 0.8, cap, seed=13 + k)
            n_steps += r["steps"]
            k += 1
        cdt = time.perf_counter() - t0
        cpu[name] = {"value": n_steps * N / cdt, "unit": "spin-steps/s", "cores": 1, "kind": "port",
                     "sample": "%d steps (episodes of <= %d steps), %.1f s, one thread" % (n_steps, cap, cdt)}
    line["cpu_baseline"] = cpu["per_agent_loop"]
    line["cpu_baseline_numpy_port"] = cpu["numpy_port"]
print(json.dumps(line), flush=True)
