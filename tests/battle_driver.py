"""Battle episode driver shared by the fixture generator and the parity tests.

Test infrastructure only.  It runs the exact env-call sequence of the
reference training loop ``senario_battle.play`` (reference
examples/battle_model/senario_battle.py:41-192) against any object with the
``magent.GridWorld`` API -- the reference engine (oracle/_ref driven through the
reference's own python wrapper) when fixtures are generated, this repository's
HIP engine when they are replayed -- and records every observable output of the
hot path per step:

    get_observation (view + feature bytes), get_agent_id, set_action, step,
    get_reward, get_alive, get_pos (post-step grid state), get_num, clear_dead.

Actions come from the synthetic "rush" policy of SURVEY.md 8(d) when recording
and from the recorded fixture when replaying, so a replay is a pure function of
the engine under test.
"""
import hashlib
import math
import random

import numpy as np

MOVE_RIGHT, MOVE_LEFT = 8, 4          # move-range index for dx = +2 / -2 (Range.h:171-215)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()


# --------------------------------------------------------------------------------------
# placements
# --------------------------------------------------------------------------------------
def generate_map_positions(map_size, seed):
    """Positions of reference ``generate_map`` (senario_battle.py:8-37) under random.seed(seed).

    Returns (left_group_id, pos_left, pos_right); the reference adds the left block to
    handles[leftID] first, then the right block to handles[1-leftID]."""
    random.seed(seed)
    width = height = map_size
    init_num = map_size * map_size * 0.04
    gap = 3
    left_id = random.randint(0, 1)
    side = int(math.sqrt(init_num)) * 2
    left = [[x, y, 0] for x in range(width // 2 - gap - side, width // 2 - gap - side + side, 2)
            for y in range((height - side) // 2, (height - side) // 2 + side, 2)]
    right = [[x, y, 0] for x in range(width // 2 + gap, width // 2 + gap + side, 2)
             for y in range((height - side) // 2, (height - side) // 2 + side, 2)]
    return left_id, left, right


def block_positions(map_size, n_side):
    """Fixed two-block placement of SURVEY.md 8(d) (used at 64x64/256 and 256x256/4096)."""
    w = h = map_size
    cols = int(math.sqrt(n_side / 2))
    rows = n_side // cols
    y0 = (h - 2 * rows) // 2
    ys = range(y0, y0 + 2 * rows, 2)
    left = [[x, y, 0] for x in range(w // 2 - 3 - 2 * cols, w // 2 - 3, 2) for y in ys]
    right = [[x, y, 0] for x in range(w // 2 + 3, w // 2 + 3 + 2 * cols, 2) for y in ys]
    return left, right


# --------------------------------------------------------------------------------------
# synthetic rush policy
# --------------------------------------------------------------------------------------
def rush_policy(view, feat, rng, view2attack, attack_base, n_action, eps=0.2):
    n = view.shape[0]
    acts = np.where(feat[:, -2] < 0.5, MOVE_RIGHT, MOVE_LEFT).astype(np.int32)
    if n:
        enemy = view[:, :, :, 4] > 0
        rows, cols = np.nonzero(view2attack >= 0)             # row-major order
        chosen = np.zeros(n, dtype=bool)
        for r, c in zip(rows, cols):
            hit = enemy[:, r, c] & ~chosen
            acts[hit] = attack_base + view2attack[r, c]
            chosen |= hit
    u = rng.random_sample(n)
    rnd = rng.randint(0, n_action, size=n).astype(np.int32)
    acts = np.where(u < eps, rnd, acts).astype(np.int32)
    return acts


# --------------------------------------------------------------------------------------
# the episode loop
# --------------------------------------------------------------------------------------
def run_episode(env, handles, placement, max_steps, policy_seed=None, actions=None,
                keep_raw=True, full_obs_steps=(), on_step=None):
    """Run one episode; returns a dict of per-step records (lists, one entry per step).

    placement: list of (group_index, positions) added in order after env.reset().
    Exactly one of policy_seed (record) / actions (replay: list of per-step [a_g0, a_g1])."""
    env.reset()
    for g, pos in placement:
        env.add_agents(handles[g], method="custom", pos=pos)
    n_group = len(handles)
    rec = {k: [] for k in ("n", "sha_view", "sha_feat", "sha_ids", "sha_reward", "sha_alive",
                           "sha_pos", "num_after", "done", "actions", "ids", "reward", "alive",
                           "pos", "mean_action")}
    rec["full_obs"] = {}
    rng = np.random.RandomState(policy_seed) if actions is None else None
    n_action = env.get_action_space(handles[0])[0]
    attack_base, v2a = env.get_view2attack(handles[0])
    done = False
    step = 0
    while not done and step < max_steps:
        obs, ids = [], []
        for g in range(n_group):
            v, f = env.get_observation(handles[g])
            obs.append((v.copy(), f.copy()))
            ids.append(env.get_agent_id(handles[g]))
        acts = []
        for g in range(n_group):
            if actions is None:
                acts.append(rush_policy(obs[g][0], obs[g][1], rng, v2a, attack_base, n_action))
            else:
                acts.append(np.ascontiguousarray(actions[step][g], dtype=np.int32))
        for g in range(n_group):
            env.set_action(handles[g], acts[g])
        done = env.step()
        rewards = [env.get_reward(handles[g]) for g in range(n_group)]
        alives = [env.get_alive(handles[g]) for g in range(n_group)]
        poss = [env.get_pos(handles[g]) for g in range(n_group)]
        nums = [env.get_num(handles[g]) for g in range(n_group)]
        # mean-action pooling of the reference training loop (senario_battle.py:141)
        means = [np.mean(list(map(lambda x: np.eye(n_action)[x], acts[g])), axis=0, keepdims=True)
                 if len(acts[g]) else np.zeros((1, n_action)) for g in range(n_group)]
        rec["n"].append([len(ids[g]) for g in range(n_group)])
        rec["sha_view"].append([sha(obs[g][0]) for g in range(n_group)])
        rec["sha_feat"].append([sha(obs[g][1]) for g in range(n_group)])
        rec["sha_ids"].append([sha(ids[g]) for g in range(n_group)])
        rec["sha_reward"].append([sha(rewards[g]) for g in range(n_group)])
        rec["sha_alive"].append([sha(alives[g]) for g in range(n_group)])
        rec["sha_pos"].append([sha(poss[g]) for g in range(n_group)])
        rec["num_after"].append(nums)
        rec["done"].append(bool(done))
        rec["actions"].append([a.copy() for a in acts])
        rec["mean_action"].append(means)
        if keep_raw:
            rec["ids"].append(ids)
            rec["reward"].append(rewards)
            rec["alive"].append(alives)
            rec["pos"].append(poss)
        if step in full_obs_steps:
            rec["full_obs"][step] = obs
        if on_step is not None:
            on_step(step, obs, acts, rewards, alives, poss, done)
        env.clear_dead()
        step += 1
    return rec


def placement_generate_map(map_size, seed):
    left_id, left, right = generate_map_positions(map_size, seed)
    return [(left_id, left), (1 - left_id, right)]


def placement_blocks(map_size, n_side):
    left, right = block_positions(map_size, n_side)
    return [(0, left), (1, right)]
