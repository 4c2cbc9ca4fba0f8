"""Per-call step time of the generic engine configs: the drop-in GridWorld on one library,
one env, the reference call sequence (get_observation of every group, set_action with random actions, step,
get_reward / get_alive, clear_dead), timed per env.step() and per whole step, after a warmup.

    python scripts/bench_generic.py --lib build/libmagent.so --config double_attack --map 24 --counts 40,60"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))

ap = argparse.ArgumentParser()
ap.add_argument("--lib", required=True)
ap.add_argument("--config", default="double_attack")
ap.add_argument("--map", type=int, default=24)
ap.add_argument("--counts", default="40,60")
ap.add_argument("--steps", type=int, default=400)
ap.add_argument("--warmup", type=int, default=50)
ap.add_argument("--seed", type=int, default=3)
a = ap.parse_args()

import numpy as np  # noqa: E402
import common  # noqa: E402

counts = [int(x) for x in a.counts.split(",")]


def mode_config(map_size, big, turn=True, food=False):
    """turn / food mode with 1x1 (big=False) or 2x3 hunters (tests/test_rules_gpu.py's _mode_config)."""
    import magent
    gw = magent.gridworld
    cfg = gw.Config()
    cfg.set({"map_width": map_size, "map_height": map_size, "turn_mode": turn, "food_mode": food,
             "minimap_mode": False, "embedding_size": 6})
    hunter = cfg.register_agent_type("hunter", dict(
        width=2 if big else 1, length=3 if big else 1, hp=6, speed=1.5, view_range=gw.CircleRange(3),
        attack_range=gw.CircleRange(1.5), damage=2, step_recover=0.1, eat_ability=1.5, food_supply=2.5, kill_reward=3,
        attack_penalty=-0.1, step_reward=-0.01))
    prey = cfg.register_agent_type("prey", dict(
        width=1, length=1, hp=4, speed=1, view_range=gw.SectorRange(3, 120), attack_range=gw.CircleRange(1),
        damage=1, step_recover=-0.02, eat_ability=0.4, food_supply=1.2, kill_supply=1.0, dead_penalty=-1))
    g0, g1 = cfg.add_group(hunter), cfg.add_group(prey)
    x, y = gw.AgentSymbol(g0, "any"), gw.AgentSymbol(g1, "any")
    cfg.add_reward_rule(gw.Event(x, "attack", y), receiver=[x, y], value=[0.2, -0.2])
    return cfg


MODES = {"turn": (False, True, False), "turn_big": (True, True, False), "food": (False, False, True),
         "turn_food": (False, True, True)}
config = mode_config(a.map, *MODES[a.config]) if a.config in MODES else a.config
env, handles = common.config_env(a.lib, config, a.map)
env.set_seed(a.seed)
rs = np.random.RandomState(a.seed)
step_t, whole_t, attackers = [], [], []


def reset():
    env.reset()
    env.add_walls(method="random", n=a.map)
    for h, n in zip(handles, counts):
        env.add_agents(h, method="random", n=n)


reset()
for t in range(a.warmup + a.steps):
    t0 = time.perf_counter()
    for h in handles:
        env.get_observation(h)
    n_att = 0
    for h in handles:
        n_act = env.get_action_space(h)[0]
        acts = rs.randint(0, n_act, env.get_num(h)).astype(np.int32)
        env.set_action(h, acts)
    t1 = time.perf_counter()
    done = env.step()
    t2 = time.perf_counter()
    for h in handles:
        env.get_reward(h)
        env.get_alive(h)
    env.clear_dead()
    t3 = time.perf_counter()
    if t >= a.warmup:
        step_t.append(t2 - t1)
        whole_t.append(t3 - t0)
    if done or min(env.get_num(h) for h in handles) == 0:
        reset()
print(json.dumps({"lib": os.path.basename(a.lib), "config": a.config, "map": a.map, "counts": counts,
                  "steps": a.steps, "step_us_median": float(np.median(step_t)) * 1e6,
                  "step_us_mean": float(np.mean(step_t)) * 1e6, "whole_us_median": float(np.median(whole_t)) * 1e6}))
