"""The drop-in single-env path (magent.GridWorld over the HIP engine, host numpy buffers, the
reference's own call sequence) timed exactly like bench.py's cpu_baseline: env calls only, the numpy
rush policy outside the clock.  Prints agent-steps/s for the HIP drop-in and, when built, the C oracle and the
reference engine itself (oracle/_ref, one OpenMP thread) through the same python wrapper, and the reference
engine driven by plain ctypes calls in the reference wrapper's pattern (no checked-call layer); hip_vs_ref is
against the faster of the two.

    python scripts/bench_dropin.py [--map 64 --agents 256 --seconds 5]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (binds the engine to torch's HIP runtime)
import battle_driver as bd  # noqa: E402
import magent  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--map", type=int, default=64)
ap.add_argument("--agents", type=int, default=256)
ap.add_argument("--seconds", type=float, default=5.0)
ap.add_argument("--calls", action="store_true", help="also report the time per call kind (us per step)")
ap.add_argument("--pause-us", type=float, default=0.0, help="host pause per step outside the clock (a slow policy)")
a = ap.parse_args()


class Clock:
    """Per-call-kind accumulator: clock.t(kind, fn, *args) times one env call."""
    def __init__(self):
        self.acc = {}

    def t(self, kind, fn, *args):
        t0 = time.perf_counter()
        r = fn(*args)
        self.acc[kind] = self.acc.get(kind, 0.0) + time.perf_counter() - t0
        return r


def run(lib_path, per_call=None):
    ck = Clock()
    env = magent.GridWorld("battle", map_size=a.map, lib=magent.load_library(lib_path))
    h = env.get_handles()
    _, v2a = env.get_view2attack(h[0])
    left, right = bd.block_positions(a.map, a.agents // 2)
    rng = np.random.RandomState(0)
    clock, steps_n, n_steps = 0.0, 0, 0
    while clock < a.seconds:
        env.reset()
        env.add_agents(h[0], method="custom", pos=left)
        env.add_agents(h[1], method="custom", pos=right)
        done, k = False, 0
        while not done and k < 400 and clock < a.seconds:
            t = time.perf_counter()
            obs = [ck.t("get_observation", env.get_observation, h[g]) for g in range(2)]
            for g in range(2):
                ck.t("get_agent_id", env.get_agent_id, h[g])
            clock += time.perf_counter() - t
            acts = [bd.rush_policy(obs[g][0], obs[g][1], rng, v2a, 13, 21) for g in range(2)]
            if a.pause_us:
                t_end = time.perf_counter() + a.pause_us * 1e-6
                while time.perf_counter() < t_end:
                    pass
            t = time.perf_counter()
            for g in range(2):
                ck.t("set_action", env.set_action, h[g], acts[g])
            done = ck.t("step", env.step)
            for g in range(2):
                ck.t("get_reward", env.get_reward, h[g])
                ck.t("get_alive", env.get_alive, h[g])
            ck.t("clear_dead", env.clear_dead)
            clock += time.perf_counter() - t
            steps_n += len(obs[0][0]) + len(obs[1][0])
            k += 1
            n_steps += 1
    if per_call is not None:
        per_call.update({kk: round(1e6 * v / n_steps, 2) for kk, v in ck.acc.items()})
    return steps_n / clock


def run_plain(lib_path, per_call=None):
    """The same loop with the reference wrapper's FFI pattern on a C engine: plain ctypes calls on the library,
    no checked-call layer (gridworld.py: get_num before every getter, env_get_observation into reused buffers,
    env_set_action / env_step / env_get_reward / env_get_info / gridworld_clear_dead).  The env is set up
    through magent.GridWorld; only the per-step calls are timed."""
    import ctypes
    ck = Clock()
    env = magent.GridWorld("battle", map_size=a.map, lib=magent.load_library(lib_path))
    L, game = env._lib.dll, env.game
    h = [x.value for x in env.get_handles()]
    _, v2a = env.get_view2attack(env.get_handles()[0])
    left, right = bd.block_positions(a.map, a.agents // 2)
    rng = np.random.RandomState(0)
    fp = ctypes.POINTER(ctypes.c_float)
    obs_bufs = {}

    def num(g):
        n = ctypes.c_int32()
        L.env_get_info(game, g, b"num", ctypes.byref(n))
        return n.value

    def get_observation(g):
        n = num(g)
        view = obs_bufs.get((g, 0))
        if view is None or view.shape[0] != n:
            view = obs_bufs[(g, 0)] = np.empty((n,) + env.view_space[g], dtype=np.float32)
            obs_bufs[(g, 1)] = np.empty((n,) + env.feature_space[g], dtype=np.float32)
        feat = obs_bufs[(g, 1)]
        bufs = (fp * 2)()
        bufs[0] = view.ctypes.data_as(fp)
        bufs[1] = feat.ctypes.data_as(fp)
        L.env_get_observation(game, g, bufs)
        return view, feat

    def info(g, name, dtype):
        buf = np.empty((num(g),), dtype=dtype)
        L.env_get_info(game, g, name, buf.ctypes.data_as(ctypes.c_void_p))
        return buf

    def get_reward(g):
        buf = np.empty((num(g),), dtype=np.float32)
        L.env_get_reward(game, g, buf.ctypes.data_as(fp))
        return buf

    def set_action(g, acts):
        acts = np.ascontiguousarray(acts)
        L.env_set_action(game, g, acts.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))

    def step():
        done = ctypes.c_int32()
        L.env_step(game, ctypes.byref(done))
        return bool(done.value)

    clock, steps_n, n_steps = 0.0, 0, 0
    while clock < a.seconds:
        env.reset()
        env.add_agents(env.get_handles()[0], method="custom", pos=left)
        env.add_agents(env.get_handles()[1], method="custom", pos=right)
        done, k = False, 0
        while not done and k < 400 and clock < a.seconds:
            t = time.perf_counter()
            obs = [ck.t("get_observation", get_observation, h[g]) for g in range(2)]
            for g in range(2):
                ck.t("get_agent_id", info, h[g], b"id", np.int32)
            clock += time.perf_counter() - t
            acts = [bd.rush_policy(obs[g][0], obs[g][1], rng, v2a, 13, 21) for g in range(2)]
            t = time.perf_counter()
            for g in range(2):
                ck.t("set_action", set_action, h[g], acts[g])
            done = ck.t("step", step)
            for g in range(2):
                ck.t("get_reward", get_reward, h[g])
                ck.t("get_alive", info, h[g], b"alive", np.bool_)
            ck.t("clear_dead", L.gridworld_clear_dead, game)
            clock += time.perf_counter() - t
            steps_n += len(obs[0][0]) + len(obs[1][0])
            k += 1
            n_steps += 1
    if per_call is not None:
        per_call.update({kk: round(1e6 * v / n_steps, 2) for kk, v in ck.acc.items()})
    return steps_n / clock


pc_hip, pc_c, pc_r, pc_p = {}, {}, {}, {}
out = {"map": a.map, "agents": a.agents, "hip_dropin": run(None, pc_hip)}
oracle = os.path.join(REPO, "oracle", "build", "libbattle_oracle.so")
if os.path.exists(oracle):
    out["c_oracle_1thread"] = run(oracle, pc_c)
ref = os.path.join(REPO, "oracle", "_ref", "libmagent_ref.so")      # the reference engine built from its sources
if os.path.exists(ref):
    import common
    common.pin_ref_threads()                                          # one OpenMP thread (its attack loop)
    out["ref_1thread"] = run(ref, pc_r)
    out["ref_plain_ctypes_1thread"] = run_plain(ref, pc_p)
    # against the faster of the two ways of driving the reference engine
    out["hip_vs_ref"] = out["hip_dropin"] / max(out["ref_1thread"], out["ref_plain_ctypes_1thread"])
if a.calls:
    out["us_per_step"] = {"hip_dropin": pc_hip, "c_oracle_1thread": pc_c, "ref_1thread": pc_r,
                          "ref_plain_ctypes_1thread": pc_p}
print(json.dumps(out))
