"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference's replay buffers.

Follows examples/battle_model/algo/tools.py (TensorFlow is only imported there, the buffers are
numpy): MetaBuffer ring append (:26-70), AgentMemory (:176-215) as a per-agent ring of sub_len
rows, MemoryGroup push / tight / sample / get_batch_num (:218-362), EpisodesBuffer push order
(:118-173).  The product buffers (mfrl_amd.algo.tools) keep the rows on the device; these keep
them in numpy lists and must produce the same batches from the same np.random stream.
PARITY UNPINNED against the reference itself (its module imports tensorflow, absent here)."""
import numpy as np


class Ring:
    """MetaBuffer: rows appended at a cursor that wraps; length saturates at max_len."""

    def __init__(self, shape, max_len, dtype):
        self.data = np.zeros((max_len,) + tuple(shape), dtype=dtype)
        self.max_len, self.flag, self.length = max_len, 0, 0

    def append(self, rows):
        rows = np.asarray(rows, dtype=self.data.dtype)
        if len(rows) > self.max_len:                  # row by row, only the last max_len would remain
            for k in range(len(rows)):
                self.append(rows[k:k + 1])
            return
        n, cut = len(rows), 0
        if self.flag + n > self.max_len:
            cut = self.max_len - self.flag
            self.data[self.flag:] = rows[:cut]
            n -= cut
            self.flag = 0
        self.data[self.flag:self.flag + n] = rows[cut:]
        self.flag += n
        self.length = min(self.length + len(rows), self.max_len)

    def pull(self):
        return self.data[:self.length]

    def sample(self, idx):
        return self.data[idx % self.length]


class MemoryGroupOracle:
    FIELDS = ("obs", "feat", "act", "rew", "term", "prob")

    def __init__(self, obs_shape, feat_shape, act_n, max_len, batch_size, sub_len, use_mean):
        self.obs_shape, self.feat_shape, self.act_n = tuple(obs_shape), tuple(feat_shape), act_n
        self.sub_len, self.batch_size, self.use_mean = sub_len, batch_size, use_mean
        spec = {"obs": (obs_shape, np.float32), "feat": (feat_shape, np.float32), "act": ((), np.int32),
                "rew": ((), np.float32), "term": ((), bool), "mask": ((), bool), "prob": ((act_n,), np.float32)}
        self.rings = {k: Ring(s, max_len, d) for k, (s, d) in spec.items()}
        self.agents = {}                                  # id -> per-agent rings, insertion order
        self.new_add = 0

    def _agent_rings(self):
        return {"obs": Ring(self.obs_shape, self.sub_len, np.float32), "feat": Ring(self.feat_shape, self.sub_len, np.float32),
                "act": Ring((), self.sub_len, np.int32), "rew": Ring((), self.sub_len, np.float32),
                "term": Ring((), self.sub_len, bool), "prob": Ring((self.act_n,), self.sub_len, np.float32)}

    def push(self, ids, obs, feat, acts, rewards, alives, prob=None):
        for i, key in enumerate(ids):
            r = self.agents.setdefault(int(key), self._agent_rings())
            r["obs"].append(obs[i:i + 1])
            r["feat"].append(feat[i:i + 1])
            r["act"].append(np.array([acts[i]], np.int32))
            r["rew"].append(np.array([rewards[i]], np.float32))
            r["term"].append(np.array([not alives[i]]))
            if self.use_mean:
                r["prob"].append(prob[i:i + 1])

    def tight(self):
        keys = list(self.agents.keys())
        np.random.shuffle(keys)
        for k in keys:
            r = self.agents[k]
            term = r["term"].pull()
            mask = ~term
            mask[-1] = False
            for f in ("obs", "feat", "act", "rew", "term"):
                self.rings[f].append(r[f].pull())
            if self.use_mean:
                self.rings["prob"].append(r["prob"].pull())
            self.rings["mask"].append(mask)
            self.new_add += len(term)
        self.agents = {}

    def sample(self):
        nb = self.rings["obs"].length
        idx = np.random.choice(nb, size=self.batch_size)
        nxt = (idx + 1) % nb
        g = lambda f, i: self.rings[f].sample(i)
        out = {"obs": g("obs", idx), "obs_next": g("obs", nxt), "feat": g("feat", idx), "feat_next": g("feat", nxt),
               "act": g("act", idx), "rew": g("rew", idx), "done": g("term", idx), "mask": g("mask", idx)}
        if self.use_mean:
            out["prob"], out["prob_next"] = g("prob", idx), g("prob", nxt)
        return out

    def get_batch_num(self):
        res = self.new_add * 2 // self.batch_size
        self.new_add = 0
        return res


def episodes_order(pushes):
    """EpisodesBuffer: agents in dict insertion order, where each push inserts in the order of
    np.random.permutation(len(view)); returns [(id, [rows as (push index, row index)])]."""
    entries = {}
    for p, ids in enumerate(pushes):
        index = np.random.permutation(len(ids))
        for i in range(len(ids)):
            j = index[i]
            entries.setdefault(int(ids[j]), []).append((p, j))
    return list(entries.items())
