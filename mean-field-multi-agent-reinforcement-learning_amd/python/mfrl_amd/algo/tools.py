"""Replay buffers and the self-play runner of algo/tools.py, with every buffer resident in HBM.

* MetaBuffer   (tools.py:26-70): fixed-size ring of rows on the GPU, same append / wrap / sample.
* MemoryGroup  (tools.py:218-362): per-agent sequences collected during an episode, flushed by
               tight() in a shuffled agent order into the rings, masks = not terminal and not the
               last row of an agent's sequence; sample() draws batch indices like the reference.
               Rows are kept step-major on the device; tight() is one gather.
* EpisodesBuffer (tools.py:118-173): rows of every agent for the AC losses, grouped per agent in
               the order the reference's dict would hold them.
* Runner       (tools.py:482-651): play one round, self-play update r = (1 - tau) l + tau r when the
               main model wins, save both models.

np.random is consumed exactly where the reference consumes it (agent shuffle, sample indices,
push permutation), so a seeded run draws the same indices.  Keys are int64 agent ids (the batched
engine passes env * cap + id).

Every row move -- a push into the episode's step rows, tight()'s gather into the rings (with their wrap),
sample()'s gather of a minibatch, EpisodesBuffer's per-agent gather -- is ONE launch of the HIP kernel
k_rows_copy (mfrl_amd.replay.rows_copy, csrc/replay_kernels.hip) over all the columns it moves; torch
computes only the index lists.  device='cpu' runs the same moves with torch indexing (the CPU tests of the
semantics against the reference's fixtures; never a fallback for a missing library on the GPU).
"""
import json
import os

import numpy as np
import torch

from .. import replay


class Color:
    INFO = "\033[1;34m{}\033[0m"
    WARNING = "\033[1;33m{}\033[0m"
    ERROR = "\033[1;31m{}\033[0m"


def _dev(x, dtype, device="cuda"):
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=dtype)
    return torch.as_tensor(np.asarray(x), dtype=dtype, device=device)


def _move(dst, src, idx=None, src_mod=0, dst_start=0, dst_cap=0, n=None, shift_mask=0, shift=0):
    """rows_copy on the device (one HIP launch for every column); torch indexing for device='cpu'.  Columns k
    with bit k of shift_mask set read row idx + shift."""
    if dst[0].is_cuda:
        assert all(d.is_contiguous() for d in dst)
        replay.rows_copy(dst, [x.contiguous() for x in src], idx, src_mod, dst_start, dst_cap, n, shift_mask, shift)
        return
    if n is None:
        n = len(idx) if idx is not None else len(src[0])
    s0 = torch.arange(n) if idx is None else idx.to(torch.int64)
    d = torch.arange(n) + dst_start
    if dst_cap:
        d = d % dst_cap
    for k, (a, b) in enumerate(zip(dst, src)):
        s = s0 + shift if shift_mask >> k & 1 else s0
        a[d] = b[s % src_mod if src_mod else s]


def ring_append(bufs, srcs, idx=None):
    """Append rows (srcs[k][idx], or srcs[k] in order) to MetaBuffers bufs[k], which share one position
    (they are always appended together), in one move: only the last max_len rows survive, the ring wraps."""
    n = len(idx) if idx is not None else len(srcs[0])
    if n == 0:
        return
    b0 = bufs[0]
    M = b0.max_len
    start, skip = b0._flag, 0
    if n > M:                                   # only the last max_len rows survive in the ring
        skip = n - M
        start = (start + skip) % M
    if idx is not None:
        idx = idx[skip:]
    else:
        srcs = [x[skip:] for x in srcs]
    _move([b.data for b in bufs], srcs, idx, dst_start=start, dst_cap=M, n=n - skip)
    for b in bufs:
        b._flag = (start + n - skip) % M
        b.length = min(b.length + n, M)


class MetaBuffer:
    def __init__(self, shape, max_len, dtype=torch.float32, device="cuda"):
        self.max_len = max_len
        self.device = device
        self.data = torch.zeros((max_len,) + tuple(shape), dtype=dtype, device=device)
        self.start = 0
        self.length = 0
        self._flag = 0

    def __len__(self):
        return self.length

    def sample(self, idx):
        out = torch.empty((len(idx),) + tuple(self.data.shape[1:]), dtype=self.data.dtype, device=self.device)
        _move([out], [self.data], idx, src_mod=self.length)
        return out

    def pull(self):
        return self.data[:self.length]

    def append(self, value):
        ring_append([self], [_dev(value, self.data.dtype, self.device)])


class _StepRows:
    """Rows pushed during an episode, step-major, on the device (grown geometrically)."""

    def __init__(self, obs_shape, feat_shape, act_n, use_mean, device="cuda"):
        self.obs_shape, self.feat_shape, self.act_n, self.use_mean = tuple(obs_shape), tuple(feat_shape), act_n, use_mean
        self.device = device
        self.n = 0
        self.cap = 0
        self.cols = {}

    def _ensure(self, need):
        if need <= self.cap:
            return
        cap = max(need, 2 * self.cap, 1024)
        spec = {"ids": ((), torch.int64), "obs": (self.obs_shape, torch.float32), "feat": (self.feat_shape, torch.float32),
                "act": ((), torch.int32), "rew": ((), torch.float32), "term": ((), torch.bool)}
        if self.use_mean:
            spec["prob"] = ((self.act_n,), torch.float32)
        new = {k: torch.empty((cap,) + s, dtype=d, device=self.device) for k, (s, d) in spec.items()}
        if self.n:
            keys = list(self.cols)
            _move([new[k] for k in keys], [self.cols[k] for k in keys], n=self.n)
        self.cols, self.cap = new, cap

    def push(self, ids, obs, feat, act, rew, alive, prob=None, order=None):
        dv = self.device
        ids = _dev(ids, torch.int64, dv)
        m = len(ids)
        sel = None if order is None else torch.as_tensor(order, device=dv, dtype=torch.int64)
        self._ensure(self.n + m)
        keys = ["ids", "obs", "feat", "act", "rew", "term"]
        src = [ids, _dev(obs, torch.float32, dv).reshape((m,) + self.obs_shape),
               _dev(feat, torch.float32, dv).reshape((m,) + self.feat_shape), _dev(act, torch.int32, dv).reshape(m),
               _dev(rew, torch.float32, dv).reshape(m), ~_dev(alive, torch.bool, dv).reshape(m)]
        if self.use_mean:
            keys.append("prob")
            src.append(_dev(prob, torch.float32, dv).reshape(m, self.act_n))
        _move([self.cols[k] for k in keys], src, sel, dst_start=self.n, n=m)
        self.n += m

    def grouped(self, key_order=None):
        """Row gather index grouping rows by agent (agents in first-appearance order, or key_order),
        steps in push order; plus the per-agent segment lengths and the agent keys."""
        ids = self.cols["ids"][:self.n]
        uniq, first = _first_appearance(ids)
        dv = self.device
        if key_order is not None:
            uniq = uniq[torch.as_tensor(key_order, device=dv, dtype=torch.int64)]
        rank = torch.empty(int(uniq.max().item()) + 1 if len(uniq) else 1, dtype=torch.int64, device=dv)
        rank[uniq] = torch.arange(len(uniq), device=dv)
        r = rank[ids]
        order = torch.argsort(r * (self.n + 1) + torch.arange(self.n, device=dv))
        counts = torch.bincount(r, minlength=len(uniq))
        return order, counts, uniq

    def clear(self):
        self.n = 0


def _first_appearance(ids):
    """Unique ids in order of first appearance (the reference's dict insertion order)."""
    if len(ids) == 0:
        return ids, ids
    uniq, inv = torch.unique(ids, return_inverse=True)
    first = torch.full((len(uniq),), len(ids), dtype=torch.int64, device=ids.device)
    first.scatter_reduce_(0, inv, torch.arange(len(ids), device=ids.device), reduce="amin")
    o = torch.argsort(first)
    return uniq[o], first[o]


class MemoryGroup:
    def __init__(self, obs_shape, feat_shape, act_n, max_len, batch_size, sub_len, use_mean=False, device="cuda"):
        self.max_len = max_len
        self.device = device
        self.batch_size = batch_size
        self.obs_shape = tuple(obs_shape)
        self.feat_shape = tuple(feat_shape)
        self.sub_len = sub_len
        self.use_mean = use_mean
        self.act_n = act_n
        self.obs0 = MetaBuffer(obs_shape, max_len, device=device)
        self.feat0 = MetaBuffer(feat_shape, max_len, device=device)
        self.actions = MetaBuffer((), max_len, dtype=torch.int32, device=device)
        self.rewards = MetaBuffer((), max_len, device=device)
        self.terminals = MetaBuffer((), max_len, dtype=torch.bool, device=device)
        self.masks = MetaBuffer((), max_len, dtype=torch.bool, device=device)
        if use_mean:
            self.prob = MetaBuffer((act_n,), max_len, device=device)
        self._new_add = 0
        self._rows = _StepRows(obs_shape, feat_shape, act_n, use_mean, device)

    def push(self, **kwargs):
        self._rows.push(kwargs["ids"], kwargs["state"][0], kwargs["state"][1], kwargs["acts"], kwargs["rewards"],
                        kwargs["alives"], kwargs.get("prob") if self.use_mean else None)

    def tight(self):
        rows = self._rows
        if rows.n == 0:
            return
        uniq, _ = _first_appearance(rows.cols["ids"][:rows.n])
        perm = list(range(len(uniq)))
        np.random.shuffle(perm)                       # the reference shuffles its agent-id list
        order, counts, _ = rows.grouped(key_order=perm)
        # AgentMemory is a ring of sub_len rows per agent and pull() returns it in slot order: row k of
        # an agent lands in slot k % sub_len, the last writer of a slot wins
        if int(counts.max().item()) > self.sub_len:
            start = torch.cumsum(counts, 0) - counts
            agent = torch.repeat_interleave(torch.arange(len(counts), device=self.device), counts)
            pos = torch.arange(len(order), device=self.device) - start[agent]
            keep = pos >= (counts - self.sub_len).clamp(min=0)[agent]
            key = agent[keep] * (self.sub_len + 1) + pos[keep] % self.sub_len
            order = order[keep][torch.argsort(key)]
            counts = torch.clamp(counts, max=self.sub_len)
        c = rows.cols
        # masks = not terminal and not the last row of an agent's sequence, laid out in step-row order so
        # that every column moves with the same gather
        mask = ~c["term"][:rows.n]
        mask[order[torch.cumsum(counts, 0) - 1]] = False
        bufs = [self.obs0, self.feat0, self.actions, self.rewards, self.terminals, self.masks]
        srcs = [c["obs"], c["feat"], c["act"], c["rew"], c["term"], mask]
        if self.use_mean:
            bufs.append(self.prob)
            srcs.append(c["prob"])
        ring_append(bufs, srcs, order)
        self._new_add += len(order)
        rows.clear()

    @property
    def nb_entries(self):
        return len(self.obs0)

    def sample(self):
        idx = np.random.choice(self.nb_entries, size=self.batch_size)
        idx = torch.as_tensor(idx, device=self.device)
        B = len(idx)
        cur = [self.obs0, self.feat0, self.actions, self.rewards, self.terminals, self.masks]
        nxt = [self.obs0, self.feat0]
        if self.use_mean:
            cur.append(self.prob)
            nxt.append(self.prob)
        # one move for the current columns at idx and the next-state columns at the reference's next_idx =
        # (idx + 1) % nb_entries (tools.py:241): the two rows of an entry are adjacent in the ring
        out = [torch.empty((B,) + tuple(b.data.shape[1:]), dtype=b.data.dtype, device=self.device) for b in cur + nxt]
        shift_mask = ((1 << len(nxt)) - 1) << len(cur)
        _move(out, [b.data for b in cur + nxt], idx, src_mod=self.nb_entries, shift_mask=shift_mask, shift=1)
        c, x = out[:len(cur)], out[len(cur):]
        obs, feature, actions, rewards, dones, masks = c[:6]
        obs_next, feature_next = x[:2]
        if self.use_mean:
            return obs, feature, actions, c[6], obs_next, feature_next, x[2], rewards, dones, masks
        return obs, feature, obs_next, feature_next, dones, rewards, actions, masks

    def get_batch_num(self):
        print("\n[INFO] Length of buffer and new add:", len(self.obs0), self._new_add)
        res = self._new_add * 2 // self.batch_size
        self._new_add = 0
        return res


class EpisodesBuffer:
    """One entry per agent: its rows of the episode, for the AC returns (tools.py:118-173)."""

    def __init__(self, use_mean=False, device="cuda"):
        self.use_mean = use_mean
        self.device = device
        self._rows = None

    def push(self, **kwargs):
        view, feature = kwargs["state"]
        if self._rows is None:
            v = view.shape[1:] if hasattr(view, "shape") else np.asarray(view).shape[1:]
            f = feature.shape[1:] if hasattr(feature, "shape") else np.asarray(feature).shape[1:]
            act_n = (kwargs["prob"].shape[1] if self.use_mean else 1)
            self._rows = _StepRows(v, f, act_n, self.use_mean, self.device)
        index = np.random.permutation(len(view))      # the reference inserts agents in this order
        self._rows.push(kwargs["ids"], view, feature, kwargs["acts"], kwargs["rewards"], kwargs["alives"],
                        kwargs.get("prob") if self.use_mean else None, order=index)

    def reset(self):
        self._rows = None

    def batch(self):
        """(rows dict gathered per agent, counts per agent) in dict order, or None if empty."""
        if self._rows is None or self._rows.n == 0:
            return None
        order, counts, keys = self._rows.grouped()
        names = list(self._rows.cols)
        out = [torch.empty((len(order),) + tuple(self._rows.cols[k].shape[1:]), dtype=self._rows.cols[k].dtype,
                           device=self.device) for k in names]
        _move(out, [self._rows.cols[k] for k in names], order)
        return dict(zip(names, out)), counts


class SummaryObj:
    """Scalar log (the reference writes TF summaries; here one JSON line per write)."""

    def __init__(self, log_dir, log_name, n_group=1):
        self.n_group = n_group
        self.name_set = set()
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, log_name + ".jsonl")

    def register(self, name_list):
        for name in name_list:
            if name in self.name_set:
                raise Exception("You cannot define different operations with same name: `{}`".format(name))
            self.name_set.add(name)

    def write(self, summary_dict, step):
        for key in summary_dict:
            if key not in self.name_set:
                raise Exception("Undefined operation: `{}`".format(key))
        rec = {"step": step}
        rec.update({k: (float(v) if np.isscalar(v) else [float(x) for x in v]) for k, v in summary_dict.items()})
        with open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")


class Runner:
    def __init__(self, sess, env, handles, map_size, max_steps, models, play_handle, render_every=None,
                 save_every=None, tau=None, log_name=None, log_dir=None, model_dir=None, train=False):
        self.env = env
        self.models = models
        self.max_steps = max_steps
        self.handles = handles
        self.map_size = map_size
        self.render_every = render_every or 0
        self.save_every = save_every
        self.play = play_handle
        self.model_dir = model_dir
        self.train = train
        self.tau = tau
        if self.train:
            self.summary = SummaryObj(log_name=log_name, log_dir=log_dir)
            self.summary_items = ["ave_agent_reward", "total_reward", "kill", "Sum_Reward", "Kill_Sum"]
            self.summary.register(self.summary_items)
            assert self.models[0].name_scope != self.models[1].name_scope
            assert len(self.models[0].vars) == len(self.models[1].vars)
            os.makedirs(self.model_dir, exist_ok=True)

    @torch.no_grad()
    def self_play_update(self):
        """r = (1 - tau) * l + tau * r for every variable (tools.py:566-569)."""
        for l_var, r_var in zip(self.models[0].vars, self.models[1].vars):
            r_var.copy_((1.0 - self.tau) * l_var + self.tau * r_var)

    def run(self, variant_eps, iteration, win_cnt=None):
        info = {"main": {"ave_agent_reward": 0.0, "total_reward": 0.0, "kill": 0.0},
                "opponent": {"ave_agent_reward": 0.0, "total_reward": 0.0, "kill": 0.0}}
        max_nums, nums, agent_r_records, total_rewards = self.play(
            env=self.env, n_round=iteration, map_size=self.map_size, max_steps=self.max_steps, handles=self.handles,
            models=self.models, print_every=50, eps=variant_eps,
            render=(iteration + 1) % self.render_every if self.render_every > 0 else False, train=self.train)
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            replay.check_errors()            # once per round: a replay move that met an out-of-range row index raises
        for i, tag in enumerate(["main", "opponent"]):
            info[tag]["total_reward"] = total_rewards[i]
            info[tag]["kill"] = max_nums[i] - nums[1 - i]
            info[tag]["ave_agent_reward"] = agent_r_records[i]
        if self.train:
            print("\n[INFO] {}".format(info["main"]))
            if info["main"]["total_reward"] > info["opponent"]["total_reward"]:
                print(Color.INFO.format("\n[INFO] Begin self-play Update ..."))
                self.self_play_update()
                print(Color.INFO.format("[INFO] Self-play Updated!\n"))
                print(Color.INFO.format("[INFO] Saving model ..."))
                self.models[0].save(self.model_dir + "-0", iteration)
                self.models[1].save(self.model_dir + "-1", iteration)
                self.summary.write(info["main"], iteration)
        else:
            print("\n[INFO] {0} \n {1}".format(info["main"], info["opponent"]))
            if info["main"]["kill"] > info["opponent"]["kill"]:
                win_cnt["main"] += 1
            elif info["main"]["kill"] < info["opponent"]["kill"]:
                win_cnt["opponent"] += 1
            else:
                win_cnt["main"] += 1
                win_cnt["opponent"] += 1
        return info
