"""Diagnostic: where the drop-in's env.step() time goes inside k_dropin_step (MFX_STAMPS build).

    MAGENT_LIB=.../build/libmagent_stamps.so python scripts/stamps_dropin.py [--map 40 --agents 128]
Lane 0's clock at the phase boundaries of each request (request seen, actions + install, agent
phase, record written, record published, write-back, clear_dead, observation published); prints the
median time of each phase in microseconds, and the host's env.step() time beside it."""
import argparse
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import battle_driver as bd  # noqa: E402
import magent  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--map", type=int, default=40)
ap.add_argument("--agents", type=int, default=128)
ap.add_argument("--steps", type=int, default=300)
a = ap.parse_args()
lib = magent.load_library(os.environ["MAGENT_LIB"])
buf = torch.zeros(1024 * 32, dtype=torch.int64, device="cuda")
assert lib.dll.mfx_battle_set_stamp_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
env = magent.GridWorld("battle", map_size=a.map, lib=lib)
h = env.get_handles()
_, v2a = env.get_view2attack(h[0])
left, right = bd.block_positions(a.map, a.agents // 2)
rng = np.random.RandomState(0)
env.reset()
env.add_agents(h[0], method="custom", pos=left)
env.add_agents(h[1], method="custom", pos=right)
host = []
for t in range(a.steps):
    obs = [env.get_observation(h[g]) for g in range(2)]
    for g in range(2):
        env.set_action(h[g], bd.rush_policy(obs[g][0], obs[g][1], rng, v2a, 13, 21))
    t0 = time.perf_counter()
    done = env.step()
    host.append(time.perf_counter() - t0)
    for g in range(2):
        env.get_reward(h[g])
        env.get_alive(h[g])
    env.clear_dead()
    if done:
        break
env.get_num(h[0])                      # a flushing call: the server leaves
torch.cuda.synchronize()
del env                                # the stamps build prints its host split here
st = buf.view(1024, 32).cpu().numpy().astype(np.float64)
rows = st[(st[:, 0] > 0) & (st[:, 7] > 0)][10:]
if not len(rows):                      # MFX_DROPIN_VARIANT=2 (answers without the step): echo stamps
    er = st[(st[:, 8] > 0) & (st[:, 10] > 0) & (st[:, 11] > 0)][10:]
    ratio = np.median((er[:, 26] - er[:, 24]) / np.maximum(er[:, 10] - er[:, 8], 1)) * 10.0 if len(er) else 0.0
    us = lambda i, j: round(float(np.median(er[:, j] - er[:, i])) * ratio / 1e3, 2) if len(er) else None
    print({"map": a.map, "agents": a.agents, "host_step_us_median": 1e6 * float(np.median(host[10:])),
           "poll start->exit": us(11, 12), "exit->seen": us(12, 8), "done0 publish": us(8, 9),
           "done1 publish": us(9, 10)})
    sys.exit(0)
ratio = np.median((rows[:, 23] - rows[:, 16]) / np.maximum(rows[:, 7] - rows[:, 0], 1)) * 10.0   # us per clock * 1e3
names = ["actions+install", "agent phase", "record", "publish", "write-back", "clear_dead", "observation"]
out = {"map": a.map, "agents": a.agents, "requests": int(len(rows)),
       "host_step_us_median": 1e6 * float(np.median(host[10:]))}
for i, n in enumerate(names):
    out[n] = round(float(np.median(rows[:, i + 1] - rows[:, i])) * ratio / 1e3, 2)
out["seen_to_published_us"] = round(float(np.median(rows[:, 4] - rows[:, 0])) * ratio / 1e3, 2)
print(out)
