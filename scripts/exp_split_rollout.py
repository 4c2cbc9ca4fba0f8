"""Experiment: k_rollout on E envs as H engines on H HIP streams (each E / H envs), so one engine's launch tail overlaps
another's launch -- agent-steps/s against one engine of E envs, same process, interleaved.

    python scripts/exp_split_rollout.py --envs 8192 --splits 1 2 4 --steps 256 --substeps 0"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))
ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=8192)
ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4])
ap.add_argument("--steps", type=int, default=256)
ap.add_argument("--warmup", type=int, default=64)
ap.add_argument("--substeps", type=int, nargs="+", default=[0])
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
import torch  # noqa: E402
import battle_driver as bd  # noqa: E402
from mfrl_amd.battle import BattleBatch  # noqa: E402

torch.cuda.set_device(0)
left, right = bd.block_positions(64, 128)
for rep in range(a.reps):
    for H in a.splits:
        for S in a.substeps:
            streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(H - 1)]
            engs = []
            for h in range(H):
                e = BattleBatch(64, a.envs // H, stream=streams[h])
                e.rollout_init([left, right], max_steps=400, eps=0.2, seed=1234 + 31 * h)
                e.rollout_substeps(S)
                engs.append(e)
            Sx = engs[0].get_substeps()
            for e in engs:
                e.rollout_step(400 + a.warmup)
            torch.cuda.synchronize()
            bufs = [torch.zeros(e.n_envs, dtype=torch.int64, device="cuda") for e in engs]

            def units():
                t = 0
                for e, b in zip(engs, bufs):
                    e.rollout_copy("agent_steps", b)
                    e.sync()
                    t += int(b.sum().item())
                return t
            u0 = units()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            done = 0
            while done < a.steps:
                n = min(Sx, a.steps - done)
                for e in engs:
                    e.rollout_step(n)
                done += n
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            u = units() - u0
            for e in engs:
                e.rollout_check()
            print(json.dumps({"envs": a.envs, "engines": H, "substeps": Sx, "rep": rep, "agent_steps_per_s": u / dt,
                              "frac": 4945 * u / dt / 8e12, "ms_per_step": 1e3 * dt / a.steps}), flush=True)
            del engs
            torch.cuda.synchronize()
