"""Ising lattice + tabular MF-Q on device (reference main_MFQ_Ising.py, examples/ising_model).

* ``neighbour_table(n_agents, view)``  -- the spin masks of Ising.py:_calc_mask as index lists;
* ``IsingLattice``                      -- R lattices, one env.step (spins := actions, rewards,
                                           observations, order parameter) per call;
* ``reference_stream(...)``             -- the exact numpy RandomState draws main_MFQ_Ising.py
                                           makes (initial spins, Boltzmann uniforms, act_group);
* ``run_mfq(...)``                      -- the whole MF-Q episode in ONE kernel launch per batch
                                           of replicas: bit-identical to main_MFQ_Ising.py in
                                           'reference' mode, on-device Philox in 'philox' mode;
* ``run_mfq_episodes(...)``             -- main_MFQ_Ising.py -epi E: episodes in sequence on one
                                           numpy stream.
Lattices up to 32767 agents (181 x 181); above 1024 the Q table lives in HBM (k_ising_mfq_big).
"""
import ctypes

import numpy as np

from . import check, lib


def neighbour_table(n_agents, view=1):
    """Ascending neighbour ids of every agent (spin_mask == 1 of Ising.py:7-58), [N][K] int16."""
    L = int(np.ceil(np.power(n_agents, 1.0 / 2)))
    if L * L != n_agents:
        raise ValueError("the Ising lattice needs a square number of agents")
    if n_agents > 32767:
        raise ValueError("the device lattice holds at most 32767 agents (int16 neighbour ids)")
    if 2 * view < L:
        # the mask's cross of +-1..view along the row and the column, wrapped: distinct cells when the
        # view is under half the side, so the rows below equal the mask scan (vectorised for large N)
        idx = np.arange(n_agents)
        r, c = idx // L, idx % L
        cols = []
        for d in range(1, view + 1):
            cols += [((r - d) % L) * L + c, ((r + d) % L) * L + c, r * L + (c - d) % L, r * L + (c + d) % L]
        return np.ascontiguousarray(np.sort(np.stack(cols, 1), axis=1).astype(np.int16))
    out = []
    for i in range(n_agents):
        row, col = i // L, i % L
        mask = np.zeros(n_agents, dtype=bool)
        for d in [d for d in range(-view, view + 1) if d != 0]:
            if 0 <= row + d < L:
                mask[i + L * d] = True
            if 0 <= col + d < L:
                mask[i + d] = True
        if row < view:                                          # periodic wrap (Ising.py:35-57)
            for k in range(view - row):
                mask[(L - 1 - k) * L + col] = True
        if col < view:
            for k in range(view - col):
                mask[row * L + (L - 1 - k)] = True
        if row >= L - view:
            for k in range(view - (L - 1 - row)):
                mask[k * L + col] = True
        if col >= L - view:
            for k in range(view - (L - 1 - col)):
                mask[row * L + k] = True
        out.append(np.nonzero(mask)[0])
    K = len(out[0])
    if any(len(o) != K for o in out):
        raise ValueError("irregular neighbourhood (lattice smaller than the view)")
    return np.ascontiguousarray(np.stack(out).astype(np.int16))


def reference_stream(seed, n_agents, steps, act_rate=1.0):
    """The RandomState draws of main_MFQ_Ising.py, in its order: make_world's reset (N spins,
    discarded), env.reset (N spins), then per step N Boltzmann uniforms (one random_sample each,
    via choice(2, 1, p)) and the act_group permutation (choice(N, K, replace=False))."""
    rs = np.random.RandomState(seed)
    for _ in range(n_agents):
        rs.choice(2)
    spins0 = np.array([rs.choice(2) for _ in range(n_agents)], dtype=np.uint8)
    u, mask = _draw_steps(rs, n_agents, steps, act_rate)
    return spins0, u, mask


def _pack_bits(bits, words):
    w = bits.reshape(words, 32).astype(np.uint64)
    return (w << np.arange(32, dtype=np.uint64)).sum(axis=1).astype(np.uint32)


class IsingLattice:
    """R replicas of an N-agent lattice on the GPU (mfx_ising_* C ABI)."""

    def __init__(self, n_agents, replicas=1, view=1):
        self.N, self.R = n_agents, replicas
        self.nbr = neighbour_table(n_agents, view)
        self.K = self.nbr.shape[1]
        L = lib()
        for fn in ("mfx_ising_create", "mfx_ising_destroy", "mfx_ising_set_spins", "mfx_ising_get_spins",
                   "mfx_ising_step", "mfx_ising_mfq_run"):
            getattr(L, fn).restype = ctypes.c_int
        self._h = ctypes.c_void_p()
        check(L.mfx_ising_create(replicas, n_agents, self.K, self.nbr.ctypes.data_as(ctypes.c_void_p),
                                 ctypes.byref(self._h)), "mfx_ising_create")

    def __del__(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().mfx_ising_destroy(self._h)

    def set_spins(self, spins):
        s = np.ascontiguousarray(spins, dtype=np.uint8).reshape(self.R, self.N)
        check(lib().mfx_ising_set_spins(self._h, s.ctypes.data_as(ctypes.c_void_p)), "set_spins")

    def get_spins(self):
        s = np.empty((self.R, self.N), dtype=np.uint8)
        check(lib().mfx_ising_get_spins(self._h, s.ctypes.data_as(ctypes.c_void_p)), "get_spins")
        return s

    def step(self, actions):
        """actions [R, N] -> (rewards f64 [R,N], obs u8 [R,N,K], n_up [R], order f64 [R])."""
        a = np.ascontiguousarray(actions, dtype=np.int32).reshape(self.R, self.N)
        rew = np.empty((self.R, self.N), np.float64)
        obs = np.empty((self.R, self.N, self.K), np.uint8)
        nup = np.empty(self.R, np.int32)
        order = np.empty(self.R, np.float64)
        P = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        check(lib().mfx_ising_step(self._h, P(a), P(rew), P(obs), P(nup), P(order)), "mfx_ising_step")
        return rew, obs, nup, order

    def run_mfq(self, steps, temperature, lr=0.1, decay_rate=0.99, decay_gap=2000, u=None, mask=None, seed=0):
        """Tabular MF-Q episode(s) from the current spins; u/mask [R,T,...] or None (Philox / all)."""
        P = lambda x: x.ctypes.data_as(ctypes.c_void_p) if x is not None else None  # noqa: E731
        if u is not None:
            u = np.ascontiguousarray(u, dtype=np.float64).reshape(self.R, steps, self.N)
        if mask is not None:
            mask = np.ascontiguousarray(mask, dtype=np.uint32).reshape(self.R, steps, -1)
        q = np.empty((self.R, self.N, self.K + 1, 2), np.float64)
        order = np.empty((self.R, steps), np.float64)
        nup = np.empty((self.R, steps), np.int32)
        done = np.empty(self.R, np.int32)
        check(lib().mfx_ising_mfq_run(self._h, steps, ctypes.c_double(temperature), ctypes.c_double(lr),
                                      ctypes.c_double(decay_rate), decay_gap, P(u), P(mask), ctypes.c_uint(seed),
                                      P(q), P(order), P(nup), P(done)), "mfx_ising_mfq_run")
        return {"q": q, "order": order, "n_up": nup, "steps": done, "spins": self.get_spins()}


def _draw_steps(rs, n_agents, steps, act_rate):
    """Per-step draws of main_MFQ_Ising.py from RandomState rs: N Boltzmann uniforms, the act_group."""
    u = np.empty((steps, n_agents), dtype=np.float64)
    words = (n_agents + 31) // 32
    mask = np.zeros((steps, words), dtype=np.uint32)
    k = int(act_rate * n_agents)
    bits = np.zeros(words * 32, dtype=np.uint8)
    for t in range(steps):
        u[t] = rs.random_sample(n_agents)
        grp = rs.choice(n_agents, k, replace=False)
        bits[:] = 0
        bits[grp] = 1
        mask[t] = _pack_bits(bits, words)
    return u, mask


def run_mfq_episodes(n_agents=400, temperature=0.8, steps=10000, episodes=1, lr=0.1, act_rate=1.0, decay_rate=0.99,
                     decay_gap=2000, seed=13):
    """main_MFQ_Ising.py with -epi episodes (:84-159): one RandomState over the whole run; every episode
    re-draws the spins (env.reset), restarts Q at zero and the temperature at 0.3, and runs until its
    own early stop.  An episode that stops at step s has consumed s steps of draws, so the next
    episode's stream is cut from the generator only after the device reports s."""
    lat = IsingLattice(n_agents, 1)
    rs = np.random.RandomState(seed)
    for _ in range(n_agents):                       # make_world -> reset_world (discarded)
        rs.choice(2)
    out = []
    for _ in range(episodes):
        lat.set_spins(np.array([[rs.choice(2) for _ in range(n_agents)]], dtype=np.uint8))
        ahead = np.random.RandomState()
        ahead.set_state(rs.get_state())
        u, mask = _draw_steps(ahead, n_agents, steps, act_rate)
        res = lat.run_mfq(steps, temperature, lr, decay_rate, decay_gap, u=u[None],
                          mask=mask[None] if act_rate != 1.0 else None)
        _draw_steps(rs, n_agents, int(res["steps"][0]), act_rate)     # what the episode consumed
        out.append(res)
    return out


def run_mfq(n_agents=400, temperature=0.8, steps=10000, lr=0.1, act_rate=1.0, decay_rate=0.99, decay_gap=2000,
            seed=13, mode="reference", replicas=1):
    """main_MFQ_Ising.py (one episode) on device.  mode='reference' reproduces the script's numpy
    stream bit for bit (replica r uses seed + r); mode='philox' draws on device."""
    lat = IsingLattice(n_agents, replicas)
    if mode == "reference":
        streams = [reference_stream(seed + r, n_agents, steps, act_rate) for r in range(replicas)]
        lat.set_spins(np.stack([s[0] for s in streams]))
        u = np.stack([s[1] for s in streams])
        mask = np.stack([s[2] for s in streams]) if act_rate != 1.0 else None
        return lat.run_mfq(steps, temperature, lr, decay_rate, decay_gap, u=u, mask=mask)
    rs = np.random.RandomState(seed)
    lat.set_spins(rs.randint(0, 2, size=(replicas, n_agents)))
    if act_rate != 1.0:
        raise ValueError("philox mode implements act_rate = 1.0 (every agent updates every step)")
    return lat.run_mfq(steps, temperature, lr, decay_rate, decay_gap, seed=seed)
