"""The training-loop drivers of examples/battle_model/senario_battle.py, restated.

* generate_map / play / battle: the reference's single-env loop (senario_battle.py:8-37, 55-185)
  on the drop-in magent.GridWorld, with any of this package's models (numpy in and out, as there).
* play_batched: the same loop over E envs of a BattleBatch, everything in HBM -- observations go
  from the engine's buffers straight into the policy forward, actions straight back into
  set_action, and the replay rows into the device MemoryGroup / EpisodesBuffer (SURVEY.md 8(f)
  rows 1-2).  Agent keys in the buffers are env * cap + id.
"""
import math
import random
import time

import numpy as np
import torch

from .. import mf
from ..battle import GET_ALIVE, GET_ID, GET_NUM, GET_REWARD


def block_positions(map_size, side_gap=3):
    """The two square blocks of generate_map (stride 2, init_num = 0.04 * map_size^2 per side)."""
    width = height = map_size
    side = int(math.sqrt(map_size * map_size * 0.04)) * 2
    left = [[x, y, 0] for x in range(width // 2 - side_gap - side, width // 2 - side_gap, 2)
            for y in range((height - side) // 2, (height - side) // 2 + side, 2)]
    right = [[x, y, 0] for x in range(width // 2 + side_gap, width // 2 + side_gap + side, 2)
             for y in range((height - side) // 2, (height - side) // 2 + side, 2)]
    return left, right


def generate_map(env, map_size, handles):
    left, right = block_positions(map_size)
    left_id = random.randint(0, 1)
    env.add_agents(handles[left_id], method="custom", pos=left)
    env.add_agents(handles[1 - left_id], method="custom", pos=right)


def _one_hot_mean(acts, n_action):
    return np.mean(list(map(lambda x: np.eye(n_action)[x], acts)), axis=0, keepdims=True)


def play(env, n_round, map_size, max_steps, handles, models, print_every, eps=1.0, render=False, train=False):
    """One round of self-play on one env (senario_battle.py:55-185)."""
    env.reset()
    generate_map(env, map_size, handles)
    step_ct, done, n_group = 0, False, len(handles)
    state, acts, ids = [None] * n_group, [None] * n_group, [None] * n_group
    alives, rewards = [None] * n_group, [None] * n_group
    nums = [env.get_num(h) for h in handles]
    max_nums = nums.copy()
    n_action = [env.get_action_space(handles[0])[0], env.get_action_space(handles[1])[0]]
    print("\n\n[*] ROUND #{0}, EPS: {1:.2f} NUMBER: {2}".format(n_round, eps, nums))
    mean_rewards = [[] for _ in range(n_group)]
    total_rewards = [[] for _ in range(n_group)]
    former_act_prob = [np.zeros((1, n_action[0])), np.zeros((1, n_action[1]))]
    while not done and step_ct < max_steps:
        for i in range(n_group):
            state[i] = list(env.get_observation(handles[i]))
            ids[i] = env.get_agent_id(handles[i])
        for i in range(n_group):
            former_act_prob[i] = np.tile(former_act_prob[i], (len(state[i][0]), 1))
            acts[i] = models[i].act(state=state[i], prob=former_act_prob[i], eps=eps)
        for i in range(n_group):
            env.set_action(handles[i], acts[i])
        done = env.step()
        for i in range(n_group):
            rewards[i] = env.get_reward(handles[i])
            alives[i] = env.get_alive(handles[i])
        buffer = {"state": state[0], "acts": acts[0], "rewards": rewards[0], "alives": alives[0], "ids": ids[0],
                  "prob": former_act_prob[0]}
        for i in range(n_group):
            former_act_prob[i] = _one_hot_mean(acts[i], n_action[i])
        if train:
            models[0].flush_buffer(**buffer)
        nums = [env.get_num(h) for h in handles]
        for i in range(n_group):
            sum_reward = sum(rewards[i])
            rewards[i] = sum_reward / nums[i]
            mean_rewards[i].append(rewards[i])
            total_rewards[i].append(sum_reward)
        if render:
            env.render()
        env.clear_dead()
        info = {"Ave-Reward": np.round(rewards, decimals=6), "NUM": nums}
        step_ct += 1
        if step_ct % print_every == 0:
            print("> step #{}, info: {}".format(step_ct, info))
    if train:
        models[0].train()
    for i in range(n_group):
        mean_rewards[i] = sum(mean_rewards[i]) / len(mean_rewards[i])
        total_rewards[i] = sum(total_rewards[i])
    return max_nums, nums, mean_rewards, total_rewards


def battle(env, n_round, map_size, max_steps, handles, models, print_every, eps=1.0, render=False, train=False):
    """Evaluation round (senario_battle.py:188-263): play without buffers or training."""
    return play(env, n_round, map_size, max_steps, handles, models, print_every, eps, render, train=False)


def play_batched(eng, n_round, map_size, max_steps, models, print_every=50, eps=1.0, train=False, left_id=None):
    """One round on all E envs of `eng` (a BattleBatch), device-resident end to end.

    Returns (max_nums, nums, mean_rewards, total_rewards) summed over envs, like play()."""
    E, G = eng.n_envs, 2
    eng.reset()
    left, right = block_positions(map_size)
    left_id = random.randint(0, 1) if left_id is None else left_id
    eng.add_agents(left_id, left)
    eng.add_agents(1 - left_id, right)
    rowcap = max(eng.capacity(g) for g in range(G))
    rowcap = (rowcap + 3) & ~3
    v_shape = tuple(models[0].view_space)
    f_shape = tuple(models[0].feature_space)
    n_action = [m.num_actions for m in models]
    key_stride = max(eng.capacity(g) for g in range(G)) * G + 1
    dev = "cuda"
    view = [torch.empty((E, rowcap) + v_shape, device=dev) for _ in range(G)]
    feat = [torch.empty((E, rowcap) + f_shape, device=dev) for _ in range(G)]
    nums_t = [torch.empty(E, dtype=torch.int32, device=dev) for _ in range(G)]
    ids_t = [torch.empty(E * rowcap, dtype=torch.int32, device=dev) for _ in range(G)]
    acts_t = [torch.zeros(E * rowcap, dtype=torch.int32, device=dev) for _ in range(G)]
    rew_t = [torch.empty(E * rowcap, dtype=torch.float32, device=dev) for _ in range(G)]
    alive_t = [torch.empty(E * rowcap, dtype=torch.uint8, device=dev) for _ in range(G)]
    done_t = torch.zeros(E, dtype=torch.int32, device=dev)
    finished = torch.zeros(E, dtype=torch.bool, device=dev)
    former = [torch.zeros((E, n_action[g]), dtype=torch.float32, device=dev) for g in range(G)]
    rows = torch.arange(rowcap, device=dev)
    env_of_row = torch.arange(E, device=dev).repeat_interleave(rowcap)
    for g in range(G):
        eng.get(g, GET_NUM, nums_t[g], rowcap)
    max_nums = [int(nums_t[g].sum().item()) for g in range(G)]
    nums = list(max_nums)
    print("\n\n[*] ROUND #{0}, EPS: {1:.2f} NUMBER: {2} ({3} envs)".format(n_round, eps, nums, E))
    mean_rewards = [[] for _ in range(G)]
    total_rewards = [[] for _ in range(G)]
    step_ct = 0
    t_play = time.time()
    agent_steps = 0
    while step_ct < max_steps and not bool(finished.all().item()):
        valid = []
        for g in range(G):
            eng.observe(g, view[g], feat[g], rowcap)
            eng.get(g, GET_NUM, nums_t[g], rowcap)
            eng.get(g, GET_ID, ids_t[g], rowcap)
            valid.append(((rows[None, :] < nums_t[g][:, None].long()) & ~finished[:, None]).reshape(-1))
        for g in range(G):
            sel = valid[g].nonzero().reshape(-1)
            prob = former[g][env_of_row[sel]]
            a = models[g].act_dev(state=[view[g].reshape((-1,) + v_shape)[sel], feat[g].reshape((-1,) + f_shape)[sel]],
                                  prob=prob, eps=eps)
            acts_t[g].zero_()
            acts_t[g][sel] = a
            eng.set_action(g, acts_t[g], rowcap)
        eng.step(done_t)
        for g in range(G):
            eng.get(g, GET_REWARD, rew_t[g], rowcap)
            eng.get(g, GET_ALIVE, alive_t[g], rowcap)
        sel0 = valid[0].nonzero().reshape(-1)
        agent_steps += int(valid[0].sum().item()) + int(valid[1].sum().item())
        if train:
            keys = env_of_row[sel0].long() * key_stride + ids_t[0][sel0].long()
            models[0].flush_buffer(state=[view[0].reshape((-1,) + v_shape)[sel0], feat[0].reshape((-1,) + f_shape)[sel0]],
                                   acts=acts_t[0][sel0], rewards=rew_t[0][sel0], alives=alive_t[0][sel0].bool(),
                                   ids=keys, prob=former[0][env_of_row[sel0]])
        for g in range(G):        # former_act_prob: mean one-hot over the env's agents (HIP kernel)
            counts = torch.where(finished, torch.zeros_like(nums_t[g]), nums_t[g])
            former[g] = mf.mean_action(acts_t[g].reshape(E, rowcap), counts, n_action[g]).float()
            former[g] = torch.nan_to_num(former[g], nan=0.0)
        for g in range(G):
            live = valid[g]
            sum_reward = float(rew_t[g][live].sum().item())
            n = int(live.sum().item())
            mean_rewards[g].append(sum_reward / max(n, 1))
            total_rewards[g].append(sum_reward)
        nums = [int(nums_t[g][~finished].sum().item()) for g in range(G)]
        eng.clear_dead()
        finished |= done_t.bool()
        step_ct += 1
        if step_ct % print_every == 0:
            print("> step #{}, Ave-Reward: {}, NUM: {}".format(step_ct, np.round([m[-1] for m in mean_rewards], 6), nums))
    torch.cuda.synchronize()
    t_play = time.time() - t_play
    t_train = time.time()
    if train:
        models[0].train()
        torch.cuda.synchronize()
    print("[TIME] play {} steps x {} envs: {:.2f} s ({:.3g} agent-steps/s incl. policy forward); train {:.2f} s"
          .format(step_ct, E, t_play, agent_steps / max(t_play, 1e-9), time.time() - t_train))
    for g in range(G):
        mean_rewards[g] = sum(mean_rewards[g]) / max(len(mean_rewards[g]), 1)
        total_rewards[g] = sum(total_rewards[g])
    return max_nums, nums, mean_rewards, total_rewards
