"""Oracle replay of sampled envs of a fused rollout (test infrastructure).

A BattleBatch rollout (k_rollout, k_rollout_bigq, or the pipelines) runs the reference training-loop
step of senario_battle.play (:96-171) on every env with the on-device rush policy.  Its actions are a
pure function of the env state, the policy seed, the env index and the step index (the counter hash of
csrc/battle/rollout.inc:9-49), so any env of the batch can be replayed on the C oracle
(oracle/battle_oracle.c, pinned to the reference engine) from rollout_init on, without reading the
device's per-step actions: `device_rush_actions` restates the device policy on the observation the
oracle returns.  After any number of launches the device's buffers for that env must then equal the
replay's, bit for bit:

* the last step's observation (views, features of every group), actions, rewards and mean action;
* the state after it (ids, positions, hp of every group member, the group sizes);
* the env's counters: agent-steps, episode statistics [episodes, return g0, return g1, kills] and the
  running episode return -- the float sums restated in the device's summation order (`device_sum`).

Used by the parity tests (tests/test_rollout_gpu.py) after every launch of the bench's own shapes, and
by bench.py after its timed region (the bench line's "check"), never inside a timed region.
"""
import numpy as np

import battle_driver as bd
import common

_U32 = np.uint32


def mix32(h):
    """murmur3 finalizer on uint32 arrays (csrc/battle/rollout.inc:9-12)."""
    h = np.asarray(h, dtype=np.uint32).copy()
    with np.errstate(over="ignore"):
        h ^= h >> _U32(16)
        h *= _U32(0x85EBCA6B)
        h ^= h >> _U32(13)
        h *= _U32(0xC2B2AE35)
        h ^= h >> _U32(16)
    return h


def policy_keys(seed, env, step, ids, group):
    """Per-agent policy key of the device rush policy (rollout.inc agent_phase / rollout_big.inc
    big_env_step): seed ^ mix32(step * 0x9E3779B9 + env * 0x632BE5AB) ^ mix32(id * 0x85EBCA77 + group)."""
    with np.errstate(over="ignore"):
        e = np.array([(step * 0x9E3779B9 + env * 0x632BE5AB) & 0xFFFFFFFF], dtype=np.uint32)
        ekey = _U32(seed & 0xFFFFFFFF) ^ mix32(e)[0]
        a = np.asarray(ids, dtype=np.uint32) * _U32(0x85EBCA77) + _U32(group)
    return ekey ^ mix32(a)


def device_rush_actions(view, feat, ids, group, env, step, seed, eps, v2a, attack_base, n_action):
    """The on-device synthetic rush policy (rollout.inc rush_action) on the host: attack
    the first attack cell (view2attack order) holding an enemy, else advance 2 cells toward the centre
    (move 8 when x / W < 0.5, else 4); with probability eps a uniform action from the counter hash."""
    n = len(ids)
    acts = np.where(feat[:, -2] < np.float32(0.5), bd.MOVE_RIGHT, bd.MOVE_LEFT).astype(np.int64)
    if n:
        enemy = view[:, :, :, 4] > 0
        order = sorted(zip(*np.nonzero(v2a >= 0)), key=lambda rc: v2a[rc])
        chosen = np.zeros(n, dtype=bool)
        for r, c in order:
            hit = enemy[:, r, c] & ~chosen
            acts[hit] = attack_base + v2a[r, c]
            chosen |= hit
    h = mix32(policy_keys(seed, env, step, ids, group))
    u = (h >> _U32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    rnd = mix32(h ^ _U32(0x68E31DA4)) % _U32(n_action)
    return np.where(u < np.float32(eps), rnd.astype(np.int64), acts).astype(np.int32)


def _butterfly(x):
    """wave_sum: x += shfl_xor(x, o) for o = 32 .. 1 over one 64-lane wave (observe.inc:285-288)."""
    x = x.astype(np.float32).copy()
    lanes = np.arange(64)
    for o in (32, 16, 8, 4, 2, 1):
        x = (x + x[lanes ^ o]).astype(np.float32)
    return x[0]


def device_sum(r, lanes):
    """A group's reward sum in the device's order: lane l adds r[l], r[l + lanes], ... (float32), then
    the wave butterfly, then (more than one wave) the wave sums in wave order (block_sum_waves)."""
    r = np.asarray(r, dtype=np.float32)
    part = np.zeros(lanes, dtype=np.float32)
    for k in range(0, len(r), lanes):
        blk = r[k:k + lanes]
        part[:len(blk)] = (part[:len(blk)] + blk).astype(np.float32)
    waves = [_butterfly(part[w * 64:(w + 1) * 64]) for w in range(lanes // 64)]
    if lanes == 64:
        return waves[0]
    tot = np.float32(0.0)
    for w in waves:
        tot = np.float32(tot + w)
    return tot


def team_lanes(path, n_total, lanes=None):
    """Lanes that sum an env's rewards: k_rollout's wave 0 alone for <= 64 agents, else its 256-lane
    workgroup; the large-env and few-env step (k_rollout_big, k_rollout_bigq) 512 lanes.  lanes: the engine's
    own (lanes for <= 64 agents, lanes above), from BattleBatch.rollout_sum_lanes, which takes precedence."""
    if lanes is not None:
        return lanes[0] if n_total <= 64 else lanes[1]
    if path in ("k_rollout", "k_rollout_obs+k_rollout"):
        return 64 if n_total <= 64 else 256
    return 512


class EnvReplay:
    """Env `env` of a batch of E, replayed on the C oracle step by step from rollout_init."""

    def __init__(self, map_size, placement, env, E, max_steps, stagger, seed, eps, path, lib=None, lanes=None):
        self.oracle, self.h = common.battle_env(lib or common.ORACLE_LIB, map_size)
        # the reference build has no "hp" info (its hp shows only in the views): state() skips it there
        self.has_hp = lib is None or lib == common.ORACLE_LIB
        self.placement = placement
        self.e, self.seed, self.eps, self.path, self.max_steps = env, seed, eps, path, max_steps
        self.lanes = lanes
        self.G = len(self.h)
        self.n_action = self.oracle.get_action_space(self.h[0])[0]
        self.attack_base, self.v2a = self.oracle.get_view2attack(self.h[0])
        self.t = 0
        self.ep_len = env * max_steps // E if stagger else 0
        self.agent_steps = 0
        self.stats = np.zeros(4, dtype=np.float64)
        self.ep_return = np.zeros(self.G, dtype=np.float32)
        self.last = None
        self._reset()

    def _reset(self):
        self.oracle.reset()
        for g, pos in enumerate(self.placement):
            self.oracle.add_agents(self.h[g], method="custom", pos=pos)

    def advance(self, T):
        """Run the steps up to global step T (exclusive)."""
        while self.t < T:
            self._step()

    def _step(self):
        o, h = self.oracle, self.h
        obs = [tuple(x.copy() for x in o.get_observation(h[g])) for g in range(self.G)]
        ids = [o.get_agent_id(h[g]) for g in range(self.G)]
        acts = [device_rush_actions(obs[g][0], obs[g][1], ids[g], g, self.e, self.t, self.seed, self.eps, self.v2a,
                                    self.attack_base, self.n_action) for g in range(self.G)]
        n = [len(x) for x in ids]
        for g in range(self.G):
            o.set_action(h[g], acts[g])
        done = o.step()
        rew = [o.get_reward(h[g]) for g in range(self.G)]
        kills = sum(int((~o.get_alive(h[g])).sum()) for g in range(self.G))
        lanes = team_lanes(self.path, sum(n), self.lanes)
        for g in range(self.G):
            self.ep_return[g] = np.float32(self.ep_return[g] + device_sum(rew[g], lanes))
        self.stats[3] += float(kills)
        self.agent_steps += sum(n)
        o.clear_dead()
        mean = [np.bincount(acts[g], minlength=self.n_action) / n[g] if n[g] else np.full(self.n_action, np.nan)
                for g in range(self.G)]
        self.last = {"n": n, "view": [x[0] for x in obs], "feature": [x[1] for x in obs], "actions": acts,
                     "rewards": rew, "mean": mean}
        self.ep_len += 1
        if done or self.ep_len >= self.max_steps:
            self.stats[0] += 1.0
            self.stats[1] += float(self.ep_return[0])
            self.stats[2] += float(self.ep_return[1]) if self.G > 1 else 0.0
            self.ep_return[:] = 0.0
            self.ep_len = 0
            self._reset()
        self.t += 1

    def state(self):
        o, h = self.oracle, self.h
        return {"ids": [o.get_agent_id(h[g]) for g in range(self.G)],
                "pos": [o.get_pos(h[g]) for g in range(self.G)],
                "hp": [o._info_array(h[g], b"hp", (o.get_num(h[g]),), np.float32) if self.has_hp else None
                       for g in range(self.G)]}


def device_records(eng, envs):
    """The same quantities for envs `envs` of the batch, read from the engine's rollout buffers and
    (ids, positions, hp) the per-call getters."""
    import torch
    from mfrl_amd.battle import GET_HP, GET_ID, GET_POS
    E, rc, G = eng.n_envs, eng.rowcap, len(eng.handles)
    NA = eng.env.get_action_space(eng.handles[0])[0]
    vf = [int(np.prod(eng.env.get_view_space(h))) for h in eng.handles]
    ff = [eng.env.get_feature_space(h)[0] for h in eng.handles]
    pin = dict(pin_memory=True)
    k = len(envs)
    out = {"view": [torch.empty((k, rc, vf[g]), dtype=torch.float32, **pin) for g in range(G)],
           "feature": [torch.empty((k, rc, ff[g]), dtype=torch.float32, **pin) for g in range(G)],
           "actions": torch.empty((k, G, rc), dtype=torch.int32, **pin),
           "rewards": torch.empty((k, G, rc), dtype=torch.float32, **pin),
           "mean": torch.empty((k, G, NA), dtype=torch.float64, **pin),
           "stats": torch.empty((k, 4), dtype=torch.float64, **pin),
           "agent_steps": torch.empty((k,), dtype=torch.int64, **pin),
           "ep_return": torch.empty((k, G), dtype=torch.float32, **pin),
           "group_num": torch.empty((k, G), dtype=torch.int32, **pin)}
    for j, e in enumerate(envs):
        for g in range(G):
            eng.rollout_copy_at("view", out["view"][g][j], e * rc * vf[g] * 4, group=g)
            eng.rollout_copy_at("feature", out["feature"][g][j], e * rc * ff[g] * 4, group=g)
        eng.rollout_copy_at("actions", out["actions"][j], e * G * rc * 4)
        eng.rollout_copy_at("rewards", out["rewards"][j], e * G * rc * 4)
        eng.rollout_copy_at("mean_action", out["mean"][j], e * G * NA * 8)
        eng.rollout_copy_at("stats", out["stats"][j], e * 4 * 8)
        eng.rollout_copy_at("agent_steps", out["agent_steps"][j], e * 8)
        eng.rollout_copy_at("episode_return", out["ep_return"][j], e * G * 4)
        eng.rollout_copy_at("group_num", out["group_num"][j], e * G * 4)
    getters = {"ids": (GET_ID, torch.int32, 1), "pos": (GET_POS, torch.int32, 2), "hp": (GET_HP, torch.float32, 1)}
    full = {}
    for name, (what, dt, w) in getters.items():
        full[name] = []
        for g in range(G):
            buf = torch.empty((E, rc, w), dtype=dt, device="cuda")
            eng.get(g, what, buf, rc)                  # (on the engine's stream)
            full[name].append(buf)
    eng.sync()                                         # before torch reads them on its own stream
    idx = torch.tensor(envs, dtype=torch.int64, device="cuda")
    dev = {name: [b.index_select(0, idx) for b in bufs] for name, bufs in full.items()}
    rec = {key: ([x.numpy() for x in v] if isinstance(v, list) else v.numpy()) for key, v in out.items()}
    for name in getters:
        rec[name] = [x.cpu().numpy() for x in dev[name]]
    return rec


def compare(dev, j, rep, tag=""):
    """Mismatches (strings) between slot j of device_records and an EnvReplay."""
    bad = []
    last, st = rep.last, rep.state()
    G = rep.G
    if int(dev["agent_steps"][j]) != rep.agent_steps:
        bad.append("%s agent_steps %d != %d" % (tag, int(dev["agent_steps"][j]), rep.agent_steps))
    if dev["stats"][j].tobytes() != rep.stats.tobytes():
        bad.append("%s stats %s != %s" % (tag, dev["stats"][j].tolist(), rep.stats.tolist()))
    if dev["ep_return"][j].tobytes() != rep.ep_return.tobytes():
        bad.append("%s episode return %s != %s" % (tag, dev["ep_return"][j].tolist(), rep.ep_return.tolist()))
    for g in range(G):
        n = last["n"][g]
        if dev["view"][g][j, :n].tobytes() != last["view"][g].reshape(n, -1).tobytes():
            bad.append("%s group %d: view" % (tag, g))
        if dev["feature"][g][j, :n].tobytes() != last["feature"][g].tobytes():
            bad.append("%s group %d: feature" % (tag, g))
        if dev["actions"][j, g, :n].tobytes() != last["actions"][g].tobytes():
            bad.append("%s group %d: actions" % (tag, g))
        if dev["rewards"][j, g, :n].tobytes() != last["rewards"][g].tobytes():
            bad.append("%s group %d: rewards" % (tag, g))
        NA = len(last["mean"][g])
        if not np.array_equal(dev["mean"][j, g, :NA], last["mean"][g], equal_nan=True):
            bad.append("%s group %d: mean action" % (tag, g))
        m = len(st["ids"][g])
        if int(dev["group_num"][j, g]) != m:
            bad.append("%s group %d: size %d != %d" % (tag, g, int(dev["group_num"][j, g]), m))
            continue
        if dev["ids"][g][j, :m, 0].tobytes() != st["ids"][g].tobytes():
            bad.append("%s group %d: ids" % (tag, g))
        if dev["pos"][g][j, :m].tobytes() != st["pos"][g].tobytes():
            bad.append("%s group %d: positions" % (tag, g))
        if st["hp"][g] is not None and dev["hp"][g][j, :m, 0].tobytes() != st["hp"][g].tobytes():
            bad.append("%s group %d: hp" % (tag, g))
    return bad


def sample_envs(E, k):
    """k envs spread over the batch, both ends included (env E-1 has the shortest first episode)."""
    if E <= k:
        return list(range(E))
    picks = {0, E - 1} | {int(x) for x in np.linspace(0, E - 1, k)}
    return sorted(picks)[:k]


class RolloutChecker:
    """Replays `envs` of a BattleBatch on the oracle alongside the device; check(T) compares them after
    the device has run T steps since rollout_init (and the replays are advanced to T)."""

    def __init__(self, eng, map_size, placement, envs, max_steps, stagger, seed, eps, lib=None):
        self.eng, self.envs = eng, list(envs)
        self.path = eng.rollout_path()
        lanes = (eng.rollout_sum_lanes(64), eng.rollout_sum_lanes(65))
        self.replays = [EnvReplay(map_size, placement, e, eng.n_envs, max_steps, stagger, seed, eps, self.path, lib=lib,
                                  lanes=lanes) for e in self.envs]

    def check(self, T):
        eng = self.eng
        eng.rollout_check()                         # device error word / queue errors first
        dev = device_records(eng, self.envs)
        bad = []
        for j, rep in enumerate(self.replays):
            rep.advance(T)
            bad += compare(dev, j, rep, "env %d step %d:" % (self.envs[j], T))
        return bad


# --------------------------------------------------------------------------------------------------------
# the reference-recorded rollout fixture (tests/golden/battle256_rollout.npz, make_battle_fixtures.py):
# env 0 of the 256x256 bench batch under the device rush policy, recorded on the reference engine itself
# --------------------------------------------------------------------------------------------------------
class RolloutFixture:
    """Expected per-launch-boundary records of env `case["env"]` from the reference recording
    (battle256_rollout: the 256x256 bench batch; battle64_rollout: the 64x64 one).  lanes: the engine's reward-sum
    teams (BattleBatch.rollout_sum_lanes for <= 64 and > 64 agents); the recording holds the sums in every team
    order the engines use, and the running episode return follows the one the engine takes at each step."""

    def __init__(self, name="battle256_rollout", lanes=(512, 512)):
        self.case = common.manifest()["cases"][name]
        self.fx = np.load(common.GOLDEN + "/" + name + ".npz")
        self.n = self.fx["n"]
        self.acts = common.unpack_actions(self.fx, "", self.n)
        self.placement = bd.block_positions(self.case["map_size"], int(self.case["placement"].replace("blocks", "")))
        T = len(self.n)
        # running quantities of the device's counters, step by step
        self.agent_steps = np.cumsum(self.n.sum(1)).astype(np.int64)
        self.stats = np.zeros((T, 4), dtype=np.float64)
        self.ep_return = np.zeros((T, self.n.shape[1]), dtype=np.float32)
        st, ret = np.zeros(4, dtype=np.float64), np.zeros(self.n.shape[1], dtype=np.float32)
        self.restart = np.zeros(T, dtype=bool)
        for t in range(T):
            L = lanes[0] if int(self.n[t].sum()) <= 64 else lanes[1]
            ret = (ret + self.fx["rsum%d" % L][t]).astype(np.float32)
            st[3] += float((self.n[t] - self.fx["num_after"][t]).sum())
            if self.fx["done"][t] or self.fx["ep_len"][t] >= self.case["max_steps"]:
                self.restart[t] = True
                st[0] += 1.0
                st[1] += float(ret[0])
                st[2] += float(ret[1])
                ret[:] = 0.0
            self.stats[t], self.ep_return[t] = st, ret

    def compare(self, dev, j, t):
        """Mismatches between slot j of device_records (taken after global step t) and the recording."""
        fx, bad, tag = self.fx, [], "step %d:" % t
        if int(dev["agent_steps"][j]) != int(self.agent_steps[t]):
            bad.append("%s agent_steps %d != %d" % (tag, int(dev["agent_steps"][j]), int(self.agent_steps[t])))
        if dev["stats"][j].tobytes() != self.stats[t].tobytes():
            bad.append("%s stats %s != %s" % (tag, dev["stats"][j].tolist(), self.stats[t].tolist()))
        if dev["ep_return"][j].tobytes() != self.ep_return[t].tobytes():
            bad.append("%s episode return %s != %s" % (tag, dev["ep_return"][j].tolist(), self.ep_return[t].tolist()))
        for g in range(self.n.shape[1]):
            n = int(self.n[t, g])
            if bd.sha(dev["view"][g][j, :n]) != fx["sha_view"][t, g].tobytes():
                bad.append("%s group %d: view" % (tag, g))
            if bd.sha(dev["feature"][g][j, :n]) != fx["sha_feat"][t, g].tobytes():
                bad.append("%s group %d: feature" % (tag, g))
            a = self.acts[t][g]
            if dev["actions"][j, g, :n].tobytes() != a.astype(np.int32).tobytes():
                bad.append("%s group %d: actions" % (tag, g))
            if bd.sha(dev["rewards"][j, g, :n]) != fx["sha_reward"][t, g].tobytes():
                bad.append("%s group %d: rewards" % (tag, g))
            NA = dev["mean"].shape[2]
            mean = np.bincount(a, minlength=NA) / n if n else np.full(NA, np.nan)
            if not np.array_equal(dev["mean"][j, g, :NA], mean, equal_nan=True):
                bad.append("%s group %d: mean action" % (tag, g))
            m = int(dev["group_num"][j, g])
            if self.restart[t]:               # the env restarted inside the launch: the reset placement
                base = sum(len(p) for p in self.placement[:g])
                want_m = len(self.placement[g])
                ids_ok = m == want_m and np.array_equal(dev["ids"][g][j, :m, 0], np.arange(base, base + m))
                pos_ok = m == want_m and np.array_equal(dev["pos"][g][j, :m], np.asarray(self.placement[g])[:, :2])
            else:
                want_m = int(fx["num_after"][t, g])
                ids_ok = m == want_m and bd.sha(dev["ids"][g][j, :m, 0]) == fx["sha_ids_cd"][t, g].tobytes()
                pos_ok = m == want_m and bd.sha(dev["pos"][g][j, :m]) == fx["sha_pos_cd"][t, g].tobytes()
            if m != want_m:
                bad.append("%s group %d: size %d != %d" % (tag, g, m, want_m))
            elif not ids_ok:
                bad.append("%s group %d: ids" % (tag, g))
            elif not pos_ok:
                bad.append("%s group %d: positions" % (tag, g))
        return bad


def replay_records(rep):
    """An EnvReplay's last step and state in the layout of device_records (one slot), so that
    RolloutFixture.compare can check the oracle replay itself against the reference recording."""
    last, st, G = rep.last, rep.state(), rep.G
    rc = max([1] + last["n"] + [len(x) for x in st["ids"]])
    NA = len(last["mean"][0])
    out = {"agent_steps": np.array([rep.agent_steps]), "stats": rep.stats[None].copy(),
           "ep_return": rep.ep_return[None].copy(), "view": [], "feature": [],
           "actions": np.zeros((1, G, rc), np.int32), "rewards": np.zeros((1, G, rc), np.float32),
           "mean": np.zeros((1, G, NA), np.float64), "group_num": np.zeros((1, G), np.int32),
           "ids": [], "pos": []}
    for g in range(G):
        n, m = last["n"][g], len(st["ids"][g])
        out["view"].append(last["view"][g].reshape(1, n, -1))
        out["feature"].append(last["feature"][g].reshape(1, n, -1))
        out["actions"][0, g, :n] = last["actions"][g]
        out["rewards"][0, g, :n] = last["rewards"][g]
        out["mean"][0, g] = last["mean"][g]
        out["group_num"][0, g] = m
        out["ids"].append(np.asarray(st["ids"][g], np.int32).reshape(1, m, 1))
        out["pos"].append(np.asarray(st["pos"][g], np.int32).reshape(1, m, 2))
    return out
