"""Generate the mean-field algorithm fixtures from the REFERENCE's own algo/ code (build container only).

    python tests/golden/make_algo_fixtures.py

The reference's examples/battle_model/algo package (base.py, ac.py, q_learning.py, tools.py) imports
TensorFlow at module level, which this image lacks.  Nothing TensorFlow-specific runs on the lines
pinned here, so a stub ``tensorflow`` module (and a stub ``magent.gridworld`` for base.py's unused
import) lets the reference's own python execute:

* ValueNet.calc_target_q (algo/base.py:192-220), called unbound on a stand-in ``self`` whose
  ``sess.run`` returns the supplied (t_q, e_q): the MF-Q target.
* MFAC.train (algo/ac.py:283-343), unbound, on a stand-in ``self`` holding a reference
  tools.EpisodesBuffer filled by its own push(); the stand-in session returns each episode's
  bootstrap value and captures the returns the reference feeds to its train op.  NumPy-1 promotion
  (the reference's TF1 era: np.float32 * python float -> float64, so ``keep`` runs in float64 and is
  rounded to float32 only when stored into r[i]) is obtained EXACTLY by returning the bootstrap value
  as float64(value_f32): float32 -> float64 is exact and every later operation is then the same
  float64 arithmetic NumPy 1 performs.  The NEP-50 variant (float32 value, as the same lines behave
  under this image's NumPy 2) is recorded beside it.
* tools.MemoryGroup push / tight / sample and tools.EpisodesBuffer push (algo/tools.py:26-362) under
  seeded np.random: the replay rows every sample() returns and the per-agent episode order.

Output: tests/golden/algo_*.npz (numeric arrays only, no pickles).
"""
import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/examples/battle_model"


def load_reference_algo():
    sys.modules["tensorflow"] = types.ModuleType("tensorflow")           # nothing below touches tf
    mg = types.ModuleType("magent")
    mg.__path__ = []
    gw = types.ModuleType("magent.gridworld")
    gw.GridWorld = object
    mg.gridworld = gw
    sys.modules["magent"], sys.modules["magent.gridworld"] = mg, gw
    spec = importlib.util.spec_from_file_location("refalgo", os.path.join(REF, "algo", "__init__.py"),
                                                  submodule_search_locations=[os.path.join(REF, "algo")])
    pkg = importlib.util.module_from_spec(spec)
    sys.modules["refalgo"] = pkg
    spec.loader.exec_module(pkg)
    return pkg, sys.modules["refalgo.base"], sys.modules["refalgo.ac"], sys.modules["refalgo.tools"]


class _Sess:
    def __init__(self, fn):
        self.fn = fn

    def run(self, fetches, feed_dict=None):
        return self.fn(fetches, feed_dict)


def mfq_target_cases(base, rs):
    """calc_target_q on batches of 64 (q_learning.py:122-131: sampled replay rows, A = 21)."""
    out = {}
    cases = []
    for b in range(4):
        M, A = 64, 21
        e_q = rs.standard_normal((M, A)).astype(np.float32)
        t_q = (3 * rs.standard_normal((M, A))).astype(np.float32)
        rew = rs.standard_normal(M).astype(np.float32)
        done = rs.random(M) < 0.25
        if b == 1:
            e_q[0, :] = 0.5                    # all tied: first index
            e_q[1, [4, 9]] = 9.0               # tie between two maxima
            e_q[2, 7] = np.nan                 # np.argmax: the first NaN wins
            e_q[3, 0] = np.nan
            t_q[4, :] = np.float32(1e30)       # large values through the float64 product
        cases.append((e_q, t_q, rew, done))
    for b, (e_q, t_q, rew, done) in enumerate(cases):
        me = types.SimpleNamespace(obs_input="obs", feat_input="feat", act_prob_input="prob", use_mf=True,
                                   t_q="t_q", e_q="e_q", gamma=0.95)
        me.sess = _Sess(lambda fetches, feed, t=t_q, e=e_q: [t, e])
        target = base.ValueNet.calc_target_q(me, obs=np.zeros((64, 1)), feature=np.zeros((64, 1)),
                                            prob=np.zeros((64, 21), np.float32), rewards=rew, dones=done)
        assert target.dtype == np.float64
        out["b%d_eq" % b], out["b%d_tq" % b], out["b%d_r" % b], out["b%d_done" % b] = e_q, t_q, rew, done
        out["b%d_target" % b] = target
    out["n_batches"] = np.int32(len(cases))
    return out


def mfac_cases(ac, tools, rs, value_dtype):
    """MFAC.train's return loop (ac.py:301-327) on episodes pushed through the reference EpisodesBuffer.

    Views carry the agent id so the stand-in session can return that episode's bootstrap value and
    the captured feed can be mapped back to episodes."""
    np.random.seed(7)
    buf = tools.EpisodesBuffer(use_mean=True)
    n_agents, steps = 24, 60
    ids = np.arange(n_agents, dtype=np.int32) * 5 + 3
    values = {int(i): np.float32(rs.standard_normal() * 4) for i in ids}
    live = ids.copy()
    for t in range(steps):
        m = len(live)
        if m == 0:
            break
        alive = rs.random(m) > 0.03
        view = np.repeat(live.astype(np.float32)[:, None, None, None], 1, axis=1)       # (m, 1, 1, 1)
        feat = np.zeros((m, 1), np.float32)
        acts = rs.integers(0, 21, m).astype(np.int32)
        rew = (rs.standard_normal(m) * 2).astype(np.float32)                            # get_reward: f32
        prob = np.tile(rs.random(21).astype(np.float32), (m, 1))
        buf.push(state=[view, feat], acts=acts, rewards=rew, alives=alive, ids=live, prob=prob)
        live = live[alive]
    episodes = list(buf.episodes())
    captured = {}

    def run(fetches, feed):
        if isinstance(fetches, list):                        # the train step: capture the returns
            captured["reward"] = np.array(feed["reward"])
            captured["view"] = np.array(feed["view"])
            return [None, 0.0, 0.0, 0.0, np.zeros(1)]
        aid = int(np.asarray(feed["view"]).reshape(-1)[0])     # bootstrap value of this episode
        return np.array([values[aid]], dtype=value_dtype)

    me = types.SimpleNamespace(replay_buffer=buf, view_space=(1, 1, 1), feature_space=(1,), num_actions=21,
                               reward_decay=0.95, view_buf=np.empty((1, 1, 1, 1)), feature_buf=np.empty((1, 1)),
                               action_buf=np.empty(1, dtype=np.int32), reward_buf=np.empty(1, dtype=np.float32),
                               input_view="view", input_feature="feat", input_act_prob="prob", action="action",
                               reward="reward", value="value", train_op="train", pg_loss="pg", vf_loss="vf",
                               reg_loss="reg", sess=_Sess(run))
    ac.MFAC.train(me)
    # episode order and lengths as the reference concatenated them
    order = [int(ep.views[0].reshape(-1)[0]) for ep in episodes]
    lens = [len(ep.rewards) for ep in episodes]
    rewards = np.concatenate([np.array(ep.rewards, dtype=np.float32) for ep in episodes])
    return {"ids": np.array(order, np.int32), "lens": np.array(lens, np.int64), "rewards": rewards,
            "value": np.array([values[i] for i in order], np.float32), "returns": captured["reward"].astype(np.float32)}


REPLAY_V, REPLAY_F, REPLAY_A = (1, 2, 2), (5,), 21
REPLAY_CASES = [(True, 400, 5000), (False, 400, 700), (True, 7, 5000), (True, 400, 300)]


def replay_pushes(ci):
    """The pushes of replay case ci: 3 episodes of one group (ids shrink as agents die, like the real
    loop after clear_dead).  Inputs are a pure function of the seed, so only outputs are stored."""
    V, F, A = REPLAY_V, REPLAY_F, REPLAY_A
    rng = np.random.default_rng(30 + ci)
    pushes = []
    for ep in range(3):
        ids = np.arange(40, dtype=np.int64) * 3 + 5
        for t in range(25):
            if len(ids) == 0:
                break
            m = len(ids)
            alive = rng.random(m) > 0.04
            pushes.append((ep, dict(ids=ids.copy(), obs=rng.random((m,) + V, dtype=np.float32),
                                    feat=rng.random((m,) + F, dtype=np.float32),
                                    acts=rng.integers(0, A, m).astype(np.int32),
                                    rewards=rng.standard_normal(m).astype(np.float32), alives=alive,
                                    prob=rng.random((m, A), dtype=np.float32))))
            ids = ids[alive]
    return pushes


def episodes_pushes():
    V, F, A = REPLAY_V, REPLAY_F, REPLAY_A
    rng = np.random.default_rng(55)
    ids = np.arange(12, dtype=np.int64) * 7 + 1
    out = []
    while len(ids) and len(out) < 6:
        m = len(ids)
        alive = rng.random(m) > 0.1
        out.append(dict(ids=ids.copy(), obs=rng.random((m,) + V, dtype=np.float32),
                        feat=rng.random((m,) + F, dtype=np.float32), acts=rng.integers(0, A, m).astype(np.int32),
                        rewards=rng.standard_normal(m).astype(np.float32), alives=alive,
                        prob=rng.random((m, A), dtype=np.float32)))
        ids = ids[alive]
    return out


def replay_cases(tools):
    """MemoryGroup (use_mean True/False, agent rings shorter than the episode, main ring wrapping) and
    EpisodesBuffer ordering, np.random seeded before every consuming call (tight: 100 + ep; sample:
    1000 * ep + b; EpisodesBuffer pushes: 9 once)."""
    V, F, A = REPLAY_V, REPLAY_F, REPLAY_A
    out = {}
    for ci, (use_mean, sub_len, max_len) in enumerate(REPLAY_CASES):
        mg = tools.MemoryGroup(V, F, A, max_len, 64, sub_len, use_mean=use_mean)
        pushes = replay_pushes(ci)
        samples, nbatch = [], []
        for ep in range(3):
            for e, p in pushes:
                if e == ep:
                    mg.push(state=[p["obs"], p["feat"]], acts=p["acts"], rewards=p["rewards"], alives=p["alives"],
                            ids=p["ids"], prob=p["prob"])
            np.random.seed(100 + ep)
            mg.tight()
            nbatch.append(mg.get_batch_num())
            for b in range(2):
                np.random.seed(1000 * ep + b)
                samples.append(mg.sample())
        key = "c%d_" % ci
        out[key + "nbatch"] = np.array(nbatch, np.int64)
        for k, smp in enumerate(samples):
            for j, arr in enumerate(smp):
                out[key + "s%d_%d" % (k, j)] = np.asarray(arr)
        out[key + "nsample"] = np.int32(len(samples))
    eb = tools.EpisodesBuffer(use_mean=True)
    np.random.seed(9)
    for p in episodes_pushes():
        eb.push(state=[p["obs"], p["feat"]], acts=p["acts"], rewards=p["rewards"], alives=p["alives"], ids=p["ids"],
                prob=p["prob"])
    eps = list(eb.episodes())
    out["eb_counts"] = np.array([len(e.rewards) for e in eps], np.int64)
    out["eb_rewards"] = np.concatenate([np.array(e.rewards, np.float32) for e in eps])
    out["eb_obs"] = np.stack([v for e in eps for v in e.views])
    out["eb_probs"] = np.stack([v for e in eps for v in e.probs])
    out["eb_terminal"] = np.array([e.terminal for e in eps])
    return out


def main():
    pkg, base, ac, tools = load_reference_algo()
    rs = np.random.default_rng(2024)
    np.savez_compressed(os.path.join(HERE, "algo_mfq_target.npz"), **mfq_target_cases(base, rs))
    legacy = mfac_cases(ac, tools, np.random.default_rng(11), np.float64)
    nep50 = mfac_cases(ac, tools, np.random.default_rng(11), np.float32)
    assert legacy["rewards"].tobytes() == nep50["rewards"].tobytes()
    out = {k: v for k, v in legacy.items() if k != "returns"}
    out["returns_numpy1"], out["returns_nep50"] = legacy["returns"], nep50["returns"]
    np.savez_compressed(os.path.join(HERE, "algo_mfac_returns.npz"), **out)
    np.savez_compressed(os.path.join(HERE, "algo_replay.npz"), **replay_cases(tools))
    print("numpy1 vs nep50 returns differ in", int((out["returns_numpy1"] != out["returns_nep50"]).sum()),
          "of", len(out["returns_nep50"]), "entries")


if __name__ == "__main__":
    main()
