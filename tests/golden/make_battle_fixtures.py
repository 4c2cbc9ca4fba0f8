"""Generate the Battle golden fixtures from the REFERENCE engine (run in the build container).

    OMP_NUM_THREADS=1 python tests/golden/make_battle_fixtures.py

Requires /root/reference and oracle/_ref/libmagent_ref.so (``make -C oracle -f Makefile.ref``).
The reference engine is driven through the reference's OWN python wrapper
(examples/battle_model/python/magent/gridworld.py, loaded from /root/reference with its
``c_lib`` module pointed at the oracle/_ref build instead of ../../build/libmagent.so),
configured by the reference's own builtin/config/battle.py, with placements checked
against the reference's own senario_battle.generate_map.  OMP_NUM_THREADS must be 1:
the reference attack loop is racy with more threads.

Output: tests/golden/battle_*.npz (numeric arrays only, no pickles) + manifest.json.

    OMP_NUM_THREADS=1 python tests/golden/make_battle_fixtures.py battle256_rollout battle64_rollout

regenerates only the named cases (the manifest's other entries are kept).
"""
import ctypes
import importlib.util
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
import battle_driver as bd  # noqa: E402

REF = "/root/reference/examples/battle_model"
REF_LIB = os.path.join(REPO, "oracle", "_ref", "libmagent_ref.so")


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference_magent():
    assert os.environ.get("OMP_NUM_THREADS") == "1", "run with OMP_NUM_THREADS=1"
    lib = ctypes.CDLL(REF_LIB, ctypes.RTLD_GLOBAL)
    pkg = types.ModuleType("magent")
    pkg.__path__ = [os.path.join(REF, "python", "magent")]
    sys.modules["magent"] = pkg
    clib = types.ModuleType("magent.c_lib")
    clib._LIB = lib
    clib.as_float_c_array = lambda b: b.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    clib.as_int32_c_array = lambda b: b.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    clib.as_bool_c_array = lambda b: b.ctypes.data_as(ctypes.POINTER(ctypes.c_bool))
    sys.modules["magent.c_lib"] = clib
    _load("magent.environment", os.path.join(REF, "python", "magent", "environment.py"))
    gw = _load("magent.gridworld", os.path.join(REF, "python", "magent", "gridworld.py"))
    pkg.gridworld = gw
    pkg.GridWorld = gw.GridWorld
    battle_cfg = _load("refcfg_battle", os.path.join(REF, "python", "magent", "builtin", "config", "battle.py"))
    scen = _load("ref_senario_battle", os.path.join(REF, "senario_battle.py"))
    return gw, battle_cfg, scen


class _Recorder:
    """Captures what reference generate_map passes to env.add_agents."""
    def __init__(self):
        self.calls = []

    def add_agents(self, handle, method, pos):
        self.calls.append((handle, method, [list(p) for p in pos]))


def check_generate_map(scen, map_size, seed):
    import random
    rec = _Recorder()
    random.seed(seed)
    scen.generate_map(rec, map_size, [0, 1])
    placement = bd.placement_generate_map(map_size, seed)
    assert [(h, p) for h, _, p in rec.calls] == placement, "generate_map restatement mismatch"
    return placement


def pack_episode(rec, prefix, out, keep_raw):
    T = len(rec["n"])
    G = len(rec["n"][0])
    out[prefix + "n"] = np.array(rec["n"], dtype=np.int32)                      # [T,G]
    for k in ("sha_view", "sha_feat", "sha_ids", "sha_reward", "sha_alive", "sha_pos"):
        out[prefix + k] = np.frombuffer(b"".join(b for row in rec[k] for b in row),
                                        dtype=np.uint8).reshape(T, G, 32)
    out[prefix + "num_after"] = np.array(rec["num_after"], dtype=np.int32)
    out[prefix + "done"] = np.array(rec["done"], dtype=np.bool_)
    out[prefix + "actions"] = np.concatenate([a for row in rec["actions"] for a in row]).astype(np.int8)
    out[prefix + "mean_action"] = np.array([[m[0] for m in row] for row in rec["mean_action"]])
    if keep_raw:
        out[prefix + "ids"] = np.concatenate([a for row in rec["ids"] for a in row]).astype(np.int32)
        out[prefix + "reward"] = np.concatenate([a for row in rec["reward"] for a in row]).astype(np.float32)
        out[prefix + "alive"] = np.concatenate([a for row in rec["alive"] for a in row]).astype(np.bool_)
        out[prefix + "pos"] = np.concatenate([a for row in rec["pos"] for a in row]).astype(np.int32)
    for step, obs in rec["full_obs"].items():
        for g in range(G):
            out[prefix + "view_s%d_g%d" % (step, g)] = obs[g][0]
            out[prefix + "feat_s%d_g%d" % (step, g)] = obs[g][1]
    return T


def main(only=()):
    gw, battle_cfg, scen = load_reference_magent()
    manifest = {"generator": "tests/golden/make_battle_fixtures.py",
                "engine": "reference MAgent (oracle/_ref, OMP_NUM_THREADS=1) via reference gridworld.py",
                "cases": {}}
    if only:
        with open(os.path.join(HERE, "battle_manifest.json")) as f:
            manifest = json.load(f)

    def want(name):
        return not only or name in only

    def new_env(map_size):
        env = gw.GridWorld(battle_cfg.get_config(map_size))
        return env, env.get_handles()

    if want("battle40"):
        case_battle40(new_env, scen, manifest)
    if want("battle64"):
        case_battle64(new_env, manifest)
    if want("battle256"):
        case_battle256(new_env, manifest)
    if want("battle_edge16"):
        case_edge16(new_env, manifest)
    if want("battle256_seq"):
        case_battle256_seq(new_env, manifest)
    if want("battle256_rollout"):
        case_battle256_rollout(new_env, manifest)
    if want("battle64_rollout"):
        case_battle64_rollout(new_env, manifest)

    with open(os.path.join(HERE, "battle_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(manifest, indent=1))


def case_battle40(new_env, scen, manifest):
    # 1) 40x40 generate_map, three seeds; seed 0 runs two episodes in ONE env (LCG persistence)
    out = {}
    env, handles = new_env(40)
    meta = {"view_space": list(map(int, env.get_view_space(handles[0]))),
            "feature_space": list(map(int, env.get_feature_space(handles[0]))),
            "action_space": list(map(int, env.get_action_space(handles[0])))}
    ab, v2a = env.get_view2attack(handles[0])
    out["view2attack"] = v2a
    out["attack_base"] = np.array(ab, dtype=np.int32)
    episodes = []
    for ep, seed in enumerate([0, 100]):          # same env: LCG state carries over
        placement = check_generate_map(scen, 40, seed)
        rec = bd.run_episode(env, handles, placement, 400, policy_seed=seed,
                             full_obs_steps=(0, 1) if ep == 0 else ())
        T = pack_episode(rec, "e%d_" % ep, out, True)
        episodes.append({"seed": seed, "policy_seed": seed, "steps": T, "placement": "generate_map"})
    del env
    np.savez_compressed(os.path.join(HERE, "battle40_seq.npz"), **out)
    manifest["cases"]["battle40_seq"] = {"map_size": 40, "episodes": episodes, **meta,
                                        "note": "two episodes in one env (attack-shuffle LCG persists across reset)"}

    for seed in (1, 2):
        out = {}
        env, handles = new_env(40)
        placement = check_generate_map(scen, 40, seed)
        rec = bd.run_episode(env, handles, placement, 400, policy_seed=seed)
        T = pack_episode(rec, "e0_", out, True)
        del env
        np.savez_compressed(os.path.join(HERE, "battle40_s%d.npz" % seed), **out)
        manifest["cases"]["battle40_s%d" % seed] = {"map_size": 40, "episodes": [
            {"seed": seed, "policy_seed": seed, "steps": T, "placement": "generate_map"}]}



def case_battle64(new_env, manifest):
    # 2) 64x64, 128 per side (8x16 blocks) -- the headline config
    out = {}
    env, handles = new_env(64)
    placement = bd.placement_blocks(64, 128)
    rec = bd.run_episode(env, handles, placement, 400, policy_seed=7, full_obs_steps=(0,))
    T = pack_episode(rec, "e0_", out, True)
    del env
    np.savez_compressed(os.path.join(HERE, "battle64.npz"), **out)
    manifest["cases"]["battle64"] = {"map_size": 64, "episodes": [
        {"seed": None, "policy_seed": 7, "steps": T, "placement": "blocks128"}]}



def case_battle256(new_env, manifest):
    # 3) 256x256, 2048 per side -- large-map band mode; hashes only, 60 steps
    out = {}
    env, handles = new_env(256)
    placement = bd.placement_blocks(256, 2048)
    rec = bd.run_episode(env, handles, placement, 60, policy_seed=11, keep_raw=False)
    T = pack_episode(rec, "e0_", out, False)
    del env
    np.savez_compressed(os.path.join(HERE, "battle256.npz"), **out)
    manifest["cases"]["battle256"] = {"map_size": 256, "episodes": [
        {"seed": None, "policy_seed": 11, "steps": T, "placement": "blocks2048"}]}



def case_edge16(new_env, manifest):
    # 4) edge: 16x16, 1 vs 6 agents, walls; one side is wiped out -> after clear_dead the
    #    survivors' minimap channel of the empty group is 0/0 (NaN in the reference).
    out = {}
    env, handles = new_env(16)
    _, v2a = env.get_view2attack(handles[0])
    env.reset()
    env.add_walls(method="custom", pos=[(5, 5), (5, 6), (5, 7), (9, 3)])
    env.add_agents(handles[0], method="custom", pos=[(7, 7, 0)])
    env.add_agents(handles[1], method="custom",
                   pos=[(6, 7, 0), (8, 7, 0), (7, 6, 0), (7, 8, 0), (6, 6, 0), (7, 8, 0)])  # dup skipped
    steps = []
    for t in range(12):
        v0, f0 = env.get_observation(handles[0])
        v1, f1 = env.get_observation(handles[1])
        out["view0_%d" % t], out["feat0_%d" % t] = v0.copy(), f0.copy()
        out["view1_%d" % t], out["feat1_%d" % t] = v1.copy(), f1.copy()
        n0, n1 = len(v0), len(v1)
        a0 = np.full(n0, 6, dtype=np.int32)                       # group 0 stays
        # group 1 attacks the cell toward the lone agent: attack idx by relative offset
        pos1 = env.get_pos(handles[1]) if n1 else np.zeros((0, 2), np.int32)
        a1 = np.full(n1, 6, dtype=np.int32)
        for i, (x, y) in enumerate(pos1):
            dx, dy = 7 - x, 7 - y
            if max(abs(dx), abs(dy)) == 1:
                a1[i] = 13 + int(v2a[6 + dy, 6 + dx])
        out["act0_%d" % t], out["act1_%d" % t] = a0, a1
        env.set_action(handles[0], a0)
        env.set_action(handles[1], a1)
        done = env.step()
        out["rew0_%d" % t], out["rew1_%d" % t] = env.get_reward(handles[0]), env.get_reward(handles[1])
        out["done_%d" % t] = np.array(done)
        env.clear_dead()
        steps.append(t)
        if env.get_num(handles[0]) == 0:
            v1, f1 = env.get_observation(handles[1])
            out["view1_final"], out["feat1_final"] = v1.copy(), f1.copy()
            break
    del env
    np.savez_compressed(os.path.join(HERE, "battle_edge16.npz"), **out)
    manifest["cases"]["battle_edge16"] = {"map_size": 16, "steps": len(steps),
                                          "note": "custom walls, duplicate placement skipped, "
                                                  "group wiped -> NaN minimap after clear_dead"}


def case_battle256_seq(new_env, manifest):
    # 5) 256x256, 2048 per side, TWO full episodes (<= 400 steps each) in ONE env under the rush
    #    policy: the large-map band order late in a fight (thinned map, clear_dead churn) and the
    #    attack-shuffle LCG carried across an episode restart in band mode (GridWorld.cc:79-89,
    #    :437-478, :662-672).  Hashes + actions only.
    out = {}
    env, handles = new_env(256)
    placement = bd.placement_blocks(256, 2048)
    episodes = []
    for ep, pseed in enumerate((21, 22)):
        rec = bd.run_episode(env, handles, placement, 400, policy_seed=pseed, keep_raw=False)
        T = pack_episode(rec, "e%d_" % ep, out, False)
        episodes.append({"seed": None, "policy_seed": pseed, "steps": T, "placement": "blocks2048"})
    del env
    np.savez_compressed(os.path.join(HERE, "battle256_seq.npz"), **out)
    manifest["cases"]["battle256_seq"] = {"map_size": 256, "episodes": episodes,
                                          "note": "two full episodes in one env (band mode, LCG persistence)"}


def case_battle256_rollout(new_env, manifest):
    # 6) env 0 of the 256x256 bench batch (bench.py: 2048 staggered envs) -- k_rollout_bigq's reference pin
    case_rollout(new_env, manifest, "battle256_rollout", 256, 2048, E=2048)


def case_battle64_rollout(new_env, manifest):
    # 7) env 0 of the 64x64 bench batch (bench.py: 131072 staggered envs, the metric's config) -- k_rollout's
    #    reference pin; also the first env of every smaller batch (configs[3]'s 8 per GPU)
    case_rollout(new_env, manifest, "battle64_rollout", 64, 128, E=131072)


def case_rollout(new_env, manifest, name, map_size, n_side, E, seed=1234, eps=0.2, max_steps=400, episodes=2):
    # env 0 of a staggered bench batch (env 0 starts at episode length 0 for any batch size) under the DEVICE rush
    # policy (tests/rollout_check.py device_rush_actions: a counter hash of seed / env / step / id), recorded on the
    # reference engine through the reference wrapper: a fused rollout of that batch must reproduce it at every launch
    # boundary.  The reward sums are recorded in the device's orders for 64-, 256- and 512-lane teams (the engine
    # reports which team sums an env-step of n agents: BattleBatch.rollout_sum_lanes).
    import rollout_check as rck
    env, h = new_env(map_size)
    placement = bd.placement_blocks(map_size, n_side)
    G = len(h)
    n_action = int(env.get_action_space(h[0])[0])
    attack_base, v2a = env.get_view2attack(h[0])
    lanes = (64, 256, 512)
    rec = {k: [] for k in ("n", "sha_view", "sha_feat", "sha_ids", "sha_reward", "sha_alive", "sha_pos",
                           "sha_ids_cd", "sha_pos_cd", "num_after", "done", "ep_len")}
    for L in lanes:
        rec["rsum%d" % L] = []
    acts_all = []

    def reset():
        env.reset()
        for g, pos in placement:
            env.add_agents(h[g], method="custom", pos=pos)

    reset()
    t, ep, ep_len = 0, 0, 0
    while ep < episodes:
        obs = [tuple(x.copy() for x in env.get_observation(h[g])) for g in range(G)]
        ids = [env.get_agent_id(h[g]) for g in range(G)]
        acts = [rck.device_rush_actions(obs[g][0], obs[g][1], ids[g], g, 0, t, seed, eps, v2a, attack_base, n_action)
                for g in range(G)]
        for g in range(G):
            env.set_action(h[g], acts[g])
        done = env.step()
        rew = [env.get_reward(h[g]) for g in range(G)]
        rec["n"].append([len(x) for x in ids])
        rec["sha_view"].append([bd.sha(o[0]) for o in obs])
        rec["sha_feat"].append([bd.sha(o[1]) for o in obs])
        rec["sha_ids"].append([bd.sha(x) for x in ids])
        rec["sha_reward"].append([bd.sha(r) for r in rew])
        rec["sha_alive"].append([bd.sha(env.get_alive(h[g])) for g in range(G)])
        rec["sha_pos"].append([bd.sha(env.get_pos(h[g])) for g in range(G)])
        for L in lanes:
            rec["rsum%d" % L].append([rck.device_sum(r, L) for r in rew])
        rec["done"].append(bool(done))
        acts_all.append(acts)
        env.clear_dead()
        rec["sha_ids_cd"].append([bd.sha(env.get_agent_id(h[g])) for g in range(G)])
        rec["sha_pos_cd"].append([bd.sha(env.get_pos(h[g])) for g in range(G)])
        rec["num_after"].append([env.get_num(h[g]) for g in range(G)])
        ep_len += 1
        rec["ep_len"].append(ep_len)
        if done or ep_len >= max_steps:
            ep += 1
            ep_len = 0
            reset()
        t += 1
    out = {"n": np.array(rec["n"], dtype=np.int32), "num_after": np.array(rec["num_after"], dtype=np.int32),
           "done": np.array(rec["done"], dtype=np.bool_), "ep_len": np.array(rec["ep_len"], dtype=np.int32),
           "actions": np.concatenate([a for row in acts_all for a in row]).astype(np.int8)}
    for L in lanes:
        out["rsum%d" % L] = np.array(rec["rsum%d" % L], dtype=np.float32)
    for k in ("sha_view", "sha_feat", "sha_ids", "sha_reward", "sha_alive", "sha_pos", "sha_ids_cd", "sha_pos_cd"):
        out[k] = np.frombuffer(b"".join(b for row in rec[k] for b in row), dtype=np.uint8).reshape(t, G, 32)
    del env
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    manifest["cases"][name] = {
        "map_size": map_size, "placement": "blocks%d" % n_side, "steps": t, "env": 0, "n_envs": E, "seed": seed,
        "eps": eps, "max_steps": max_steps, "episodes": episodes, "sum_lanes": list(lanes),
        "note": "env 0 of the staggered bench batch under the device rush policy; per step: obs / ids / "
                "rewards / alive / pos hashes, post-clear_dead ids / pos hashes, actions, reward sums in the "
                "64-, 256- and 512-lane device orders"}


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))
