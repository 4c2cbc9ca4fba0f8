"""Diagnostic: per-phase cycle shares of k_rollout from the MFX_STAMPS build.

    MAGENT_LIB=.../build/libmagent_stamps.so python scripts/stamps_battle.py --envs 4096
Reports median / mean cycles per phase over envs for a few steady-state steps (shares only:
the stamp build's barriers forbid overlaps the real kernel has)."""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import numpy as np  # noqa: E402
import battle_driver as bd  # noqa: E402
from mfrl_amd.battle import BattleBatch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=4096)
ap.add_argument("--steps", type=int, default=5)
a = ap.parse_args()
names = ["load", "agent_count", "minimap", "obs", "policy+mean", "set_action", "step", "reward", "clear_dead",
         "episode_reset", "write_back"]
eng = BattleBatch(64, a.envs, stream=torch.cuda.current_stream())
left, right = bd.block_positions(64, 128)
eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=1)
buf = torch.zeros(a.envs * 16, dtype=torch.int64, device="cuda")
assert eng._dll.mfx_battle_set_stamp_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
eng.rollout_step(400)
torch.cuda.synchronize()
acc = []
for t in range(a.steps):
    eng.rollout_step(1)
    torch.cuda.synchronize()
    st = buf.view(a.envs, 16).cpu().numpy().astype(np.int64)
    acc.append(np.diff(st[:, :11], axis=1))
d = np.concatenate(acc)
tot = d.sum(1)
print("env lifetime (stamp 0 -> 10): median %d cycles, mean %d" % (np.median(tot), tot.mean()))
for i, n in enumerate(names[1:]):
    print("%-14s median %8d  mean %8d  share %5.1f%%" % (n, np.median(d[:, i]), d[:, i].mean(), 100 * d[:, i].mean() / tot.mean()))
