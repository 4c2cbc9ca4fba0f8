"""Diagnostic: per-phase cycle shares of k_rollout from the MFX_STAMPS build.

    MAGENT_LIB=.../build/libmagent_stamps.so python scripts/stamps_battle.py --envs 4096
Reports median / mean cycles per phase over envs for a few steady-state steps (shares only:
the stamp build's barriers forbid overlaps the real kernel has).  Shader-clock (s_memtime) deltas within one env's
processing only: the stamp build records no wall-clock (s_memrealtime) slots, so it says nothing about residency or
launch spans (scripts/timeline_rollout.py measures those)."""
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
names = ["load", "install", "minimap", "obs", "policy+mean", "set_action", "step", "reward", "clear_dead",
         "episode_reset", "write_back"]
eng = BattleBatch(64, a.envs, stream=torch.cuda.current_stream())
left, right = bd.block_positions(64, 128)
eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=1)
print("rollout grid %d workgroups, %d B dynamic LDS each" % eng.rollout_info())
buf = torch.zeros(a.envs * 32, dtype=torch.int64, device="cuda")
assert eng._dll.mfx_battle_set_stamp_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
eng.rollout_step(400)
torch.cuda.synchronize()
acc = []
raw = []
sub = []
for t in range(a.steps):
    buf.zero_()
    eng.rollout_step(1)
    torch.cuda.synchronize()
    st = buf.view(a.envs, 32).cpu().numpy().astype(np.int64)
    done = (st[:, 0] > 0) & (st[:, 10] > st[:, 0])      # envs whose stamps 0 .. 10 all landed this launch
    st = st[done]
    raw.append(st)
    acc.append(np.diff(st[:, :11], axis=1))
    sub.append(np.stack([st[:, 13] - st[:, 0], st[:, 1] - st[:, 13]], 1))
d = np.concatenate(acc)
tot = d.sum(1)
print("env lifetime (stamp 0 -> 10): median %d cycles, mean %d (%d env-steps)" % (np.median(tot), tot.mean(), len(tot)))
sb = np.concatenate(sub)
print("  install split: LDS stores + barrier mean %d cycles, prefetch issue + barrier mean %d cycles" % tuple(sb.mean(0)))
R = np.concatenate(raw)
parts = np.stack([R[:, 17] - R[:, 5], R[:, 18] - R[:, 17], R[:, 15] - R[:, 18], R[:, 19] - R[:, 15],
                  R[:, 6] - R[:, 19]], 1)
ok = (parts > 0).all(1)
for lo, hi, tag in ((0, 64, "<= 64 agents (wave team)"), (65, 10 ** 9, "> 64 agents (workgroup team)")):
    sel = ok & (R[:, 16] >= lo) & (R[:, 16] <= hi)
    if sel.any():
        print("step split, %s, %d env-steps: pre %d, attacks %d, starve %d, moves %d, rules+done %d; "
              "whole env %d" % ((tag, sel.sum()) + tuple(parts[sel].mean(0).astype(int)) +
                                (int((R[sel, 10] - R[sel, 0]).mean()),)))
        big = sel & (R[:, 26] > 0)
        if big.any():               # attack_big internals (workgroup teams): draws, buckets, positions,
            q = np.stack([R[:, 23] - R[:, 17], R[:, 24] - R[:, 23], R[:, 25] - R[:, 24],   # target buckets +
                          R[:, 26] - R[:, 25], R[:, 18] - R[:, 26]], 1)[big]               # fixed point, apply
            print("    attack_big: draws %d, shuffle buckets %d, positions %d, targets+fixed point %d, apply %d"
                  % tuple(q.mean(0).astype(int)))
for i, n in enumerate(names[1:]):
    print("%-14s median %8d  mean %8d  share %5.1f%%" % (n, np.median(d[:, i]), d[:, i].mean(), 100 * d[:, i].mean() / tot.mean()))
