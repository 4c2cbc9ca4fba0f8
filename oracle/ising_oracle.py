"""TEST ORACLE ONLY -- numpy restatement of the Ising MF-Q path (tests/, smoke() and bench.py's
cpu_baseline leg may use it; the product never does).

Restates, in vectorised numpy of its own:
  * Ising.py:_calc_mask (:7-58)               -> neighbours()
  * IsingWorld.step + Scenario.reward/observation (core.py:99-125, Ising.py:101-119) -> env_step()
  * main_MFQ_Ising.py's episode loop (:84-159) and its numpy RandomState draws -> mfq(),
    mfq_episodes() (-epi E: episodes in sequence on one stream)
Pinned bit-exactly against tests/golden/ising_*.npz, which make_ising_fixtures.py recorded by
running the reference's own Scenario / IsingWorld code.
"""
import numpy as np


def neighbours(n_agents, view=1):
    L = int(round(n_agents ** 0.5))
    assert L * L == n_agents
    idx = np.arange(n_agents)
    r, c = idx // L, idx % L
    cols = []
    for d in range(1, view + 1):
        for dr, dc in ((-d, 0), (d, 0), (0, -d), (0, d)):
            cols.append(((r + dr) % L) * L + (c + dc) % L)
    return np.sort(np.stack(cols, 1), axis=1)


def env_step(spins, nbr, actions):
    """spins/actions: [N] 0/1 -> (new spins, reward f64 [N], obs [N,K], n_up, order)."""
    s = (np.asarray(actions) > 0).astype(np.int64)
    pm = 2 * s - 1
    nsum = pm[nbr].sum(axis=1).astype(np.float64)
    reward = -((-0.5 * pm.astype(np.float64)) * nsum)
    n_up = int(s.sum())
    order = abs(n_up - (len(s) - n_up)) / (len(s) + 0.0)
    return s, reward, s[nbr], n_up, order


def mfq(n_agents, temperature, steps, lr=0.1, act_rate=1.0, decay_rate=0.99, decay_gap=2000, seed=13):
    rs = np.random.RandomState(seed)
    for _ in range(n_agents):                  # make_world -> reset_world
        rs.choice(2)
    return _episode(rs, n_agents, temperature, steps, lr, act_rate, decay_rate, decay_gap)


def mfq_episodes(n_agents, temperature, steps, episodes, lr=0.1, act_rate=1.0, decay_rate=0.99, decay_gap=2000,
                 seed=13):
    """main_MFQ_Ising.py -epi: every episode on the same RandomState (:84-159)."""
    rs = np.random.RandomState(seed)
    for _ in range(n_agents):
        rs.choice(2)
    return [_episode(rs, n_agents, temperature, steps, lr, act_rate, decay_rate, decay_gap) for _ in range(episodes)]


def _episode(rs, n_agents, temperature, steps, lr, act_rate, decay_rate, decay_gap):
    spins = np.array([rs.choice(2) for _ in range(n_agents)], dtype=np.int64)   # env.reset()
    nbr = neighbours(n_agents)
    K = nbr.shape[1]
    Q = np.zeros((n_agents, K + 1, 2))
    current_t, max_order, done_ = 0.3, 0.0, 0
    orders, nups, acts = [], [], []
    n_upd = int(act_rate * n_agents)
    ar = np.arange(n_agents)
    for t in range(steps):
        if t % decay_gap == 0:
            current_t *= decay_rate
        if current_t < temperature:
            current_t = temperature
        st = spins[nbr].sum(axis=1)
        e0 = np.exp(Q[ar, st, 0] / current_t)
        e1 = np.exp(Q[ar, st, 1] / current_t)
        denom = e0 + e1
        p0, p1 = e0 / denom, e1 / denom
        c0 = p0 / (p0 + p1)
        u = rs.random_sample(n_agents)
        action = (u >= c0).astype(np.int64)
        spins, reward, _obs, n_up, order = env_step(spins, nbr, action)
        grp = rs.choice(n_agents, n_upd, replace=False)
        Q[grp, st[grp], action[grp]] = Q[grp, st[grp], action[grp]] + lr * (reward[grp] - Q[grp, st[grp], action[grp]])
        orders.append(order)
        nups.append(n_up)
        acts.append(action)
        if order > max_order:
            max_order = order
        if abs(max_order - order) < 0.001:
            done_ += 1
        else:
            done_ = 0
        if done_ == 500:
            break
    return {"q": Q, "order": np.array(orders), "n_up": np.array(nups), "actions": np.stack(acts),
            "spins": spins, "steps": len(orders)}


def mfq_loop(n_agents, temperature, steps, lr=0.1, act_rate=1.0, decay_rate=0.99, decay_gap=2000, seed=13):
    """main_MFQ_Ising.py's episode loop (:84-159) restated PER AGENT, as the script runs it -- the CPU baseline
    of the reference loop (one core), not a faster port: boltzman_explore per agent (:55-67: np.exp per action,
    list arithmetic, np.random.choice(2, 1, p)), the env step per agent over the dense N-long spin masks
    (IsingWorld.step, Scenario.reward / observation: core.py:99-116, Ising.py:101-119, each O(N) per agent),
    and the Q update loop over act_group (:126-133).  The same numpy stream as mfq(), bit for bit
    (tests/test_ising_cpu.py)."""
    rs = np.random.RandomState(seed)
    for _ in range(n_agents):                  # make_world -> reset_world
        rs.choice(2)
    np_state = np.random.get_state()
    np.random.set_state(rs.get_state())        # the script draws from the global numpy stream
    try:
        L = int(round(n_agents ** 0.5))
        spin = [int(np.random.choice(2)) for _ in range(n_agents)]            # env.reset()
        nbr = neighbours(n_agents)
        masks = np.zeros((n_agents, n_agents))
        for i in range(n_agents):
            masks[i, nbr[i]] = 1.0
        gstate = np.array(spin, dtype=np.float64).reshape(L, L)
        obs = [gstate.flatten()[np.where(masks[i] == 1)] for i in range(n_agents)]
        Q = np.zeros((n_agents, nbr.shape[1] + 1, 2))
        current_t, max_order, done_ = 0.3, 0.0, 0
        orders = []
        for t in range(steps):
            action = np.zeros(n_agents, dtype=np.int32)
            if t % decay_gap == 0:
                current_t *= decay_rate
            if current_t < temperature:
                current_t = temperature
            for i in range(n_agents):
                obs_flat = np.count_nonzero(obs[i] == 1)
                nums, denom = [], 0
                for a in range(2):
                    val = np.exp(Q[i, obs_flat, a] / current_t)
                    nums.append(val)
                    denom += val
                action[i] = np.random.choice(2, 1, p=[x / denom for x in nums])[0]
            # IsingMultiAgentEnv._step: spins := actions, then per agent observation and reward (new spins)
            for i in range(n_agents):
                gstate[i // L, i % L] = 0 if action[i] == 0 else 1
            n_up = np.count_nonzero(gstate.flatten())
            order = abs(n_up - (n_agents - n_up)) / (n_agents + 0.0)
            obs_, reward = [], []
            for i in range(n_agents):
                obs_.append(gstate.flatten()[np.where(masks[i] == 1)])
                g = gstate.copy()
                g[np.where(g == 0)] = -1
                local = -0.5 * g[i // L, i % L] * np.sum(g.flatten() * masks[i])
                reward.append(-local)
            act_group = np.random.choice(n_agents, int(act_rate * n_agents), replace=False)
            for i in act_group:
                obs_flat = np.count_nonzero(obs[i] == 1)
                Q[i, obs_flat, action[i]] = Q[i, obs_flat, action[i]] + lr * (reward[i] - Q[i, obs_flat, action[i]])
            obs = obs_
            orders.append(order)
            if order > max_order:
                max_order = order
            if abs(max_order - order) < 0.001:
                done_ += 1
            else:
                done_ = 0
            if done_ == 500:
                break
        return {"q": Q, "order": np.array(orders), "steps": len(orders)}
    finally:
        np.random.set_state(np_state)


class MT19937Words:
    """numpy's legacy MT19937 restated word by word (numpy/random/src/mt19937/mt19937.c: init_genrand seeding of
    RandomState(seed), the 624-word twist, tempering) with the legacy draws main_MFQ_Ising.py makes, as the device
    stream (k_mt_words, k_ising_scan) consumes them: choice(2) = one word & 1; random_sample = one double from two
    words; choice(N, k, replace=False) = the legacy shuffle of arange(N), random_interval by masked rejection.
    Pure python (test infrastructure: pins that consumption model against numpy itself)."""

    def __init__(self, seed):
        k = [0] * 624
        k[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            k[i] = (1812433253 * (k[i - 1] ^ (k[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.key, self.pos, self.count = k, 624, 0

    def _twist(self):
        k = self.key
        for i in range(624):
            y = (k[i] & 0x80000000) | (k[(i + 1) % 624] & 0x7FFFFFFF)
            k[i] = k[(i + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        self.pos = 0

    def word(self):
        if self.pos >= 624:
            self._twist()
        y = self.key[self.pos]
        self.pos += 1
        self.count += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y

    def choice2(self):
        return self.word() & 1

    def random_sample(self):
        a, b = self.word() >> 5, self.word() >> 6
        return (a * 67108864.0 + b) / 9007199254740992.0

    def interval(self, mx):
        m = mx
        for s in (1, 2, 4, 8, 16):
            m |= m >> s
        while True:
            v = self.word() & m
            if v <= mx:
                return v

    def choice_no_replace(self, n, k):
        x = list(range(n))
        for i in range(n - 1, 0, -1):
            j = self.interval(i)
            x[i], x[j] = x[j], x[i]
        return x[:k]
