"""Profiling driver (run under rocprofv3): fused rollout vs the per-call kernel pipeline.

    python scripts/prof_battle.py --mode fused|percall --envs 4096 --steps 20
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import torch  # noqa: E402

import battle_driver as bd  # noqa: E402
from mfrl_amd.battle import BattleBatch, GET_REWARD, GET_ALIVE, GET_ID  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="fused")
ap.add_argument("--envs", type=int, default=4096)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--burn", type=int, default=400)
a = ap.parse_args()
torch.cuda.set_device(0)
st = torch.cuda.current_stream()
eng = BattleBatch(64, a.envs, stream=st)
left, right = bd.block_positions(64, 128)
E = a.envs
if a.mode == "fused":
    eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=1)
    eng.rollout_step(a.burn)
    torch.cuda.synchronize()
    eng.rollout_step(a.steps)
    torch.cuda.synchronize()
else:
    eng.reset()
    eng.add_agents(0, left)
    eng.add_agents(1, right)
    rc = 128
    view = [torch.empty(E * rc * 1183, device="cuda") for _ in range(2)]
    feat = [torch.empty(E * rc * 34, device="cuda") for _ in range(2)]
    acts = torch.empty(E * rc, dtype=torch.int32, device="cuda")
    rew = torch.empty(E * rc, dtype=torch.float32, device="cuda")
    ids = torch.empty(E * rc, dtype=torch.int32, device="cuda")
    alive = torch.empty(E * rc, dtype=torch.uint8, device="cuda")
    for t in range(a.steps):
        for g in range(2):
            eng.observe(g, view[g], feat[g], rc)
            eng.get(g, GET_ID, ids, rc)
        for g in range(2):
            torch.randint(0, 21, (E * rc,), out=acts)
            eng.set_action(g, acts, rc)
        eng.step()
        for g in range(2):
            eng.get(g, GET_REWARD, rew, rc)
            eng.get(g, GET_ALIVE, alive, rc)
        eng.clear_dead()
    torch.cuda.synchronize()
    eng.sync()
print("ok")
