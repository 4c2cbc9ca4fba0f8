"""Ising lattice + tabular MF-Q on the GPU (through the mfx_ising_* C ABI).

* the fused MF-Q kernel in 'reference' mode -- numpy's RandomState stream generated on the device --
  reproduces the reference trajectories recorded in tests/golden/ising_*.npz bit for bit: every action,
  order parameter, n_up, the early-stop step and the float64 Q table;
* the drop-in examples.ising_model env driven by main_MFQ_Ising.py's own loop gives the same;
* the batched env step matches the numpy oracle on random lattices (R replicas);
* Philox mode: ordered phase at low temperature, disordered at high temperature."""
import json
import os
import sys

import numpy as np
import pytest

import common

sys.path.insert(0, os.path.join(common.REPO, "oracle"))
import ising_oracle  # noqa: E402

pytestmark = pytest.mark.gpu

with open(os.path.join(common.GOLDEN, "ising_manifest.json")) as f:
    CASES = json.load(f)["cases"]


@pytest.mark.parametrize("name", sorted(CASES))
def test_fused_mfq_matches_reference(name):
    from mfrl_amd.ising import run_mfq
    c = CASES[name]
    fx = np.load(os.path.join(common.GOLDEN, name + ".npz"))
    out = run_mfq(c["n_agents"], c["temperature"], c["steps"], lr=c["lr"], act_rate=c["act_rate"], seed=c["seed"])
    T = c["stopped_after"]
    assert int(out["steps"][0]) == T
    assert out["order"][0, :T].tobytes() == fx["order"].tobytes()
    np.testing.assert_array_equal(out["n_up"][0, :T], fx["n_up"])
    np.testing.assert_array_equal(out["spins"][0], fx["spins"][-1])
    assert out["q"][0].tobytes() == fx["q_final"].tobytes()


def _main_loop_with_dropin(n_agents, temperature, steps, seed=13, lr=0.1):
    """main_MFQ_Ising.py:11-159 (one episode), unchanged apart from the step count, on the drop-in."""
    from examples.ising_model.multiagent.environment import IsingMultiAgentEnv
    import examples.ising_model as ising_model
    np.random.seed(seed)
    scen = ising_model.load("Ising.py").Scenario()
    env = IsingMultiAgentEnv(world=scen.make_world(num_agents=n_agents, agent_view=1),
                             reset_callback=scen.reset_world, reward_callback=scen.reward,
                             observation_callback=scen.observation, done_callback=scen.done)
    n_actions = env.action_space[0].n
    assert env.observation_space[0].n == 4
    obs = np.stack(env.reset())
    Q = np.zeros((env.n, 5, n_actions))
    current_t = 0.3
    acts = []
    for t in range(steps):
        action = np.zeros(env.n, dtype=np.int32)
        if t % 2000 == 0:
            current_t *= 0.99
        if current_t < temperature:
            current_t = temperature
        for i in range(env.n):
            s = np.count_nonzero(obs[i] == 1)
            vals = [np.exp(Q[i, s, k] / current_t) for k in range(n_actions)]
            denom = 0
            for v in vals:
                denom += v
            action[i] = np.random.choice(n_actions, 1, p=[v / denom for v in vals])[0]
        obs_, reward, done, order, ups, downs = env.step(np.expand_dims(action, axis=1))
        obs_ = np.stack(obs_)
        for i in np.random.choice(env.n, env.n, replace=False):
            s = np.count_nonzero(obs[i] == 1)
            Q[i, s, action[i]] = Q[i, s, action[i]] + lr * (reward[i][0] - Q[i, s, action[i]])
        obs = obs_
        acts.append(action.copy())
    return np.stack(acts), Q


def test_dropin_env_under_the_reference_loop():
    c = CASES["ising10_t05"]
    fx = np.load(os.path.join(common.GOLDEN, "ising10_t05.npz"))
    T = 120
    acts, Q = _main_loop_with_dropin(c["n_agents"], c["temperature"], T)
    np.testing.assert_array_equal(acts, fx["actions"][:T])
    q_at = list(fx["q_steps"]).index(T - 1 + 1) if (T) in list(fx["q_steps"] + 1) else None
    if q_at is not None:
        assert Q.tobytes() == fx["q"][q_at].tobytes()


def test_env_step_matches_oracle_random():
    from mfrl_amd.ising import IsingLattice
    rs = np.random.RandomState(5)
    for n, R in ((16, 3), (400, 8), (900, 2)):
        lat = IsingLattice(n, replicas=R)
        nbr = ising_oracle.neighbours(n)
        lat.set_spins(rs.randint(0, 2, size=(R, n)))
        acts = rs.randint(0, 2, size=(R, n))
        rew, obs, nup, order = lat.step(acts)
        for r in range(R):
            s, rw, ob, nu, od = ising_oracle.env_step(None, nbr, acts[r])
            assert rew[r].tobytes() == rw.tobytes()
            np.testing.assert_array_equal(obs[r], ob)
            assert nup[r] == nu and order[r] == od
        np.testing.assert_array_equal(lat.get_spins(), acts)


def test_philox_mode_phases():
    from mfrl_amd.ising import run_mfq
    cold = run_mfq(400, 0.3, 3000, mode="philox", replicas=8, seed=3)
    hot = run_mfq(400, 5.0, 600, mode="philox", replicas=8, seed=3)
    last = lambda o: np.array([o["order"][r, o["steps"][r] - 1] for r in range(8)])  # noqa: E731
    # numpy oracle, same settings, 6 seeds: cold mean 0.43 (0.04..1.0), hot mean 0.045
    assert last(cold).mean() > 0.25, last(cold)
    assert last(hot).mean() < 0.15, last(hot)
    assert last(cold).mean() > last(hot).mean() + 0.15


def test_episodes_match_reference_fixture():
    """main_MFQ_Ising.py -epi 3 on the device (run_mfq_episodes): each episode one launch, the next
    episode's stream cut after the stop step the device reports (tests/golden/ising4_epi3.npz)."""
    from mfrl_amd.ising import run_mfq_episodes
    with open(os.path.join(common.GOLDEN, "ising_manifest.json")) as f:
        c = json.load(f)["episode_cases"]["ising4_epi3"]
    fx = np.load(os.path.join(common.GOLDEN, "ising4_epi3.npz"))
    got = run_mfq_episodes(c["n_agents"], c["temperature"], c["steps"], c["episodes"], seed=c["seed"])
    for k, ep in enumerate(got):
        p = "e%d_" % k
        T = int(fx[p + "stop"])
        assert int(ep["steps"][0]) == T == c["stops"][k]
        assert ep["order"][0, :T].tobytes() == fx[p + "order"].tobytes()
        np.testing.assert_array_equal(ep["n_up"][0, :T], fx[p + "n_up"])
        assert ep["q"][0].tobytes() == fx[p + "q_final"].tobytes()


@pytest.mark.parametrize("n_agents,steps", [(1600, 60), (4096, 40), (16384, 12)])
def test_large_lattice_mfq_matches_oracle(n_agents, steps):
    """Lattices beyond one 1024-lane workgroup (k_ising_mfq_big: Q in HBM, spins in LDS) in reference
    mode against the numpy oracle: every order parameter, n_up and the float64 Q table, bit for bit."""
    from mfrl_amd.ising import run_mfq
    got = run_mfq(n_agents, 0.8, steps, seed=21)
    ref = ising_oracle.mfq(n_agents, 0.8, steps, seed=21)
    assert int(got["steps"][0]) == ref["steps"]
    assert got["order"][0, :ref["steps"]].tobytes() == ref["order"].tobytes()
    np.testing.assert_array_equal(got["n_up"][0, :ref["steps"]], ref["n_up"])
    assert got["q"][0].tobytes() == ref["q"].tobytes()


def test_large_lattice_env_step_matches_oracle():
    from mfrl_amd.ising import IsingLattice
    rs = np.random.RandomState(8)
    n, R = 32761, 2                                          # 181 x 181, the largest lattice
    lat = IsingLattice(n, replicas=R)
    nbr = ising_oracle.neighbours(n)
    np.testing.assert_array_equal(lat.nbr, nbr)
    lat.set_spins(rs.randint(0, 2, size=(R, n)))
    acts = rs.randint(0, 2, size=(R, n))
    rew, obs, nup, order = lat.step(acts)
    for r in range(R):
        s, rw, ob, nu, od = ising_oracle.env_step(None, nbr, acts[r])
        assert rew[r].tobytes() == rw.tobytes()
        np.testing.assert_array_equal(obs[r], ob)
        assert nup[r] == nu and order[r] == od


@pytest.mark.parametrize("n_agents,replicas,steps,act_rate", [(400, 6, 700, 1.0), (100, 3, 300, 0.5),
                                                              (1600, 2, 50, 1.0), (4, 5, 900, 0.75)])
def test_device_stream_matches_host_stream(n_agents, replicas, steps, act_rate):
    """numpy's RandomState stream generated on the device (k_mt_words: MT19937; k_ising_scan: the act_group
    permutation's rejection walk, the act_group bits when act_rate < 1) against the same stream drawn by numpy on
    the host and uploaded (mode 'host'): replica r = seed 13 + r; Q, every order parameter, n_up, the stop step and
    the final spins bit for bit -- including the large-lattice kernel (1600 agents) and a 2x2 lattice whose episodes
    run to the step cap."""
    from mfrl_amd.ising import run_mfq
    dev = run_mfq(n_agents, 0.8, steps, act_rate=act_rate, seed=13, replicas=replicas)
    host = run_mfq(n_agents, 0.8, steps, act_rate=act_rate, seed=13, replicas=replicas, mode="host")
    np.testing.assert_array_equal(dev["steps"], host["steps"])
    for r in range(replicas):
        T = int(host["steps"][r])
        assert dev["order"][r, :T].tobytes() == host["order"][r, :T].tobytes(), r
        np.testing.assert_array_equal(dev["n_up"][r, :T], host["n_up"][r, :T])
    assert dev["q"].tobytes() == host["q"].tobytes()
    np.testing.assert_array_equal(dev["spins"], host["spins"])


def test_device_stream_many_replicas_match_oracle():
    """2048 replicas of configs[0] (20x20, tau 0.8) on the device stream in one call (one word-generation pass):
    sampled replicas against the numpy oracle (oracle/ising_oracle.py mfq, seed 13 + r) bit for bit."""
    from mfrl_amd.ising import run_mfq
    R, T = 2048, 600
    got = run_mfq(400, 0.8, T, seed=13, replicas=R)
    for r in (0, 1, 777, R - 1):
        ref = ising_oracle.mfq(400, 0.8, T, seed=13 + r)
        assert int(got["steps"][r]) == ref["steps"]
        assert got["order"][r, :ref["steps"]].tobytes() == ref["order"].tobytes()
        assert got["q"][r].tobytes() == ref["q"].tobytes()


def test_device_stream_multi_pass_episodes_match_oracle(monkeypatch):
    """The word streams of many replicas in several generation passes (MFX_ISING_PASS_GB=1: ~119 replicas of 400
    agents x 700 steps x 2 episodes per pass, 512 replicas = 5 passes: the two-slot pipeline, pass p + 2 produced
    once pass p released its slot) with 2 episodes per replica on one stream: sampled replicas of every pass,
    both episodes, against the numpy oracle (mfq_episodes, seed 13 + r) bit for bit."""
    from mfrl_amd.ising import IsingLattice
    monkeypatch.setenv("MFX_ISING_PASS_GB", "1")
    R, T = 512, 700
    got = IsingLattice(400, R).run_mfq_stream(T, 0.8, seed=13, episodes=2)
    for r in (0, 118, 119, 300, R - 1):
        ref = ising_oracle.mfq_episodes(400, 0.8, T, 2, seed=13 + r)
        for k in range(2):
            S = ref[k]["steps"]
            assert int(got[k]["steps"][r]) == S, (r, k)
            assert got[k]["order"][r, :S].tobytes() == ref[k]["order"].tobytes(), (r, k)
            np.testing.assert_array_equal(got[k]["n_up"][r, :S], ref[k]["n_up"])
            assert got[k]["q"][r].tobytes() == ref[k]["q"].tobytes(), (r, k)


def test_device_stream_refuses_word_offsets_past_32_bits():
    """episodes x T x 4 N words per replica past 2^32 cannot be addressed by the 32-bit per-step offsets: the call
    fails loudly before any allocation, and run_mfq_episodes takes the host stream for such runs."""
    import magent
    from mfrl_amd import ising
    lat = ising.IsingLattice(400, 1)
    assert ising.stream_words(400, 10000, 300) * 1 > 2 ** 32
    with pytest.raises(magent.EngineError, match="32-bit"):
        lat.run_mfq_stream(10000, 0.8, episodes=300)
    assert 4 * ising.stream_words(400, 10000, 300) > ising.STREAM_MAX_BYTES


def test_episodes_host_fallback_matches_reference_mode(monkeypatch):
    """run_mfq_episodes past STREAM_MAX_BYTES per replica runs the host stream: the same episodes bit for bit."""
    from mfrl_amd import ising
    ref = ising.run_mfq_episodes(36, 0.8, 900, 3, seed=5)
    monkeypatch.setattr(ising, "STREAM_MAX_BYTES", 1024)
    got = ising.run_mfq_episodes(36, 0.8, 900, 3, seed=5)
    for a, b in zip(ref, got):
        assert int(a["steps"][0]) == int(b["steps"][0])
        assert a["q"].tobytes() == b["q"].tobytes()
        assert a["order"][0, :int(a["steps"][0])].tobytes() == b["order"][0, :int(b["steps"][0])].tobytes()
