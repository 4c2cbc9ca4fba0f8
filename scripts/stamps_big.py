"""Diagnostic: per-phase cycles of k_rollout_big (large envs) from the MFX_STAMPS build.

    MAGENT_LIB=.../build/libmagent_stamps.so python scripts/stamps_big.py --envs 1024
Stamps (s_memtime, shader cycles) are taken behind workgroup barriers: shares, not overlaps."""
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
ap.add_argument("--envs", type=int, default=1024)
ap.add_argument("--map", type=int, default=256)
ap.add_argument("--agents", type=int, default=4096)
ap.add_argument("--steps", type=int, default=5)
a = ap.parse_args()
names = ["policy+mean", "set_action", "fy draws", "fy buckets", "fy positions", "tgt buckets+fixed point",
         "attack apply", "starve+band sort", "moves", "rules+done", "reward", "clear_dead", "restart", "obs prep"]
eng = BattleBatch(a.map, a.envs, stream=torch.cuda.current_stream())
left, right = bd.block_positions(a.map, a.agents // 2)
eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=1)
buf = torch.zeros(a.envs * 32, dtype=torch.int64, device="cuda")
assert eng._dll.mfx_battle_set_stamp_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
eng.rollout_step(400)
torch.cuda.synchronize()
acc = []
for t in range(a.steps):
    buf.zero_()
    eng.rollout_step(1)
    torch.cuda.synchronize()
    st = buf.view(a.envs, 32).cpu().numpy().astype(np.int64)
    st = st[st[:, 8] > 0]                       # envs whose moves ran in parallel (all stamps present)
    acc.append(np.diff(st[:, :15], axis=1))
d = np.concatenate(acc)
tot = d.sum(1)
print("k_rollout_big per env: median %d cycles, mean %d (%d env-steps)" % (np.median(tot), tot.mean(), len(d)))
for i, n in enumerate(names):
    print("%-18s median %8d  mean %8d  share %5.1f%%" % (n, np.median(d[:, i]), d[:, i].mean(),
                                                       100 * d[:, i].mean() / tot.mean()))
