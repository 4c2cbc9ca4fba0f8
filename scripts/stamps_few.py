"""Diagnostic: per-phase cycles of the pipelined few-env stepper (k_rollout_bigq<true>, MFX_STAMPS build).

    MAGENT_LIB=.../build/libmagent_stamps.so python scripts/stamps_few.py --envs 8 --sub 20

Each launch runs --sub steps; row e + E k holds env e's step k of the launch (the write-back of the env to HBM
after the launch's last step is outside the stamps).  Stamps (s_memtime, shader clock) sit behind workgroup
barriers: shares, not overlaps; slots 30 / 31 hold the 100 MHz real-time clock at the step's start / end, so the
shader clock is measured rather than assumed."""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import battle_driver as bd  # noqa: E402
from mfrl_amd.battle import BattleBatch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=8)
ap.add_argument("--map", type=int, default=64)
ap.add_argument("--agents", type=int, default=256)
ap.add_argument("--sub", type=int, default=20)
ap.add_argument("--launches", type=int, default=40)
ap.add_argument("--snap", action="store_true", help="also the snapshot's sub-phases (slots 24-27)")
a = ap.parse_args()
# slot order along one step: snapshot, wait + file, then few_env_step (agent_phase's team stamps, the episode end)
order = [20, 21, 22, 4, 5, 17, 18, 15, 19, 6, 7, 8, 13]
names = ["snapshot+minimap", "wait items+file", "policy+mean", "set_action", "step prologue", "attacks",
         "starve+move order", "moves", "rules+done", "reward", "clear_dead", "episode end+restart"]
eng = BattleBatch(a.map, a.envs, stream=torch.cuda.current_stream())
left, right = bd.block_positions(a.map, a.agents // 2)
eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=1)
eng.rollout_substeps(a.sub)
buf = torch.zeros(a.envs * a.sub * 32, dtype=torch.int64, device="cuda")
assert eng._dll.mfx_battle_set_stamp_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
eng.rollout_step(200)
torch.cuda.synchronize()
acc, skipped, agents, real, gaps, snap_rows = [], 0, [], [], [], []
for t in range(a.launches):
    buf.zero_()
    eng.rollout_step(a.sub)
    torch.cuda.synchronize()
    raw3 = buf.view(a.sub, a.envs, 32).cpu().numpy().astype(np.int64)
    gaps.append((raw3[1:, :, 30] - raw3[:-1, :, 31]).ravel())     # real-time ticks between a step's end and the next
    raw = raw3.reshape(a.sub * a.envs, 32)
    snap_rows.append(raw.copy())
    st = raw[:, order]
    ok = (st > 0).all(1)                 # rows whose every stamp ran (moves in parallel, pipelined stepper)
    skipped += int((~ok).sum())
    acc.append(np.diff(st[ok], axis=1))
    agents.append(raw[ok, 16])
    real.append(raw[ok, 31] - raw[ok, 30])
eng.rollout_check()
d = np.concatenate(acc)
nag = np.concatenate(agents)
rt = np.concatenate(real) * 0.01                    # us (100 MHz)
gp = np.concatenate(gaps) * 0.01
tot = d.sum(1)
clk = tot.sum() / rt.sum() / 1e3                    # GHz
print("pipelined stepper, %d envs of %dx%d, %d agents, every step of %d-step launches: median %d cycles, mean %d "
      "(%d env-steps, %d rows without every stamp); real time per step median %.2f us, mean %.2f us -> shader clock "
      "%.2f GHz; between steps median %.2f us" % (a.envs, a.map, a.map, a.agents, a.sub, np.median(tot), tot.mean(),
                                                   len(d), skipped, np.median(rt), rt.mean(), clk, np.median(gp)))
for i, n in enumerate(names):
    print("%-24s median %8d  mean %8d  share %5.1f%%" % (n, np.median(d[:, i]), d[:, i].mean(),
                                                         100 * d[:, i].mean() / tot.mean()))
if a.snap:
    # the snapshot's sub-phases (slots 24-27, the first copying lane's clock, no barriers): from the step's start
    # (slot 20) to the copy's start, the cells, the id arrays and lists, the minimap counts + info words, then the
    # barrier's exit (slot 21)
    R = np.concatenate(snap_rows)
    sel = (R[:, 16] <= 64) & (R[:, [20, 24, 25, 26, 27, 21]] > 0).all(1)
    q = np.diff(R[sel][:, [20, 24, 25, 26, 27, 21]], axis=1)
    print("snapshot split (<= 64 agents, %d env-steps), medians: to copy start %d, copies %d, (none) %d, "
          "counts+info %d, barrier %d" % ((int(sel.sum()),) + tuple(int(x) for x in np.median(q, 0))))
    # the policy phase of the wave team (slots 22 -> 9 -> 10 -> 11 -> 23 -> 28 -> 4): to few_agents, its views and
    # psync, agent_phase's entry, ahist zero + psync, the policy loop, the mean action
    cols = [22, 9, 10, 11, 23, 28, 4]
    sel = (R[:, 16] <= 64) & (R[:, cols] > 0).all(1)
    q = np.diff(R[sel][:, cols], axis=1)
    print("policy split (<= 64 agents, %d env-steps), medians: to few_agents %d, views+psync %d, agent_phase entry %d, "
          "ahist zero %d, policy loop %d, mean action %d" % ((int(sel.sum()),) + tuple(int(x) for x in np.median(q, 0))))
for lab, m in (("<= 64 agents", nag <= 64), ("65-128 agents", (nag > 64) & (nag <= 128)), ("> 128 agents", nag > 128)):
    if m.any():
        print("%s: %d env-steps, median %d cycles per step; phase medians %s" % (
            lab, int(m.sum()), np.median(tot[m]), " ".join("%d" % np.median(d[m, i]) for i in range(len(names)))))
# attack_big's internals on the workgroup team's steps (slots 17 -> 0 -> 1 -> 2 -> 3 -> 18, stamps build, > 64 agents):
# the Fisher-Yates draws, the shuffle buckets, the positions + targets, the target buckets + fixed point, the apply
R = np.concatenate(snap_rows)
cols = [17, 0, 1, 2, 3, 18]
for lab, lo, hi in (("65-128 agents", 65, 128), ("> 128 agents", 129, 10 ** 9)):
    sel = (R[:, 16] >= lo) & (R[:, 16] <= hi) & (R[:, cols] > 0).all(1)
    if sel.any():
        q = np.diff(R[sel][:, cols], axis=1)
        print("attack_big split (%s, %d env-steps), medians: draws %d, shuffle buckets %d, positions+targets %d, "
              "target buckets+fixed point %d, apply %d" % ((lab, int(sel.sum())) + tuple(int(x) for x in np.median(q, 0))))
