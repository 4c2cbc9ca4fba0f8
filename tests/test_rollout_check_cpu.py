"""The host side of the rollout replays (tests/rollout_check.py) on the CPU: the restated device rush
policy, the device summation order, and a replay driving the C oracle.  Their agreement with the device
itself is what tests/test_rollout_gpu.py and the bench's self-check establish on the GPU."""
import numpy as np

import battle_driver as bd
import common
import rollout_check as rck


def _mix32_py(h):
    h &= 0xFFFFFFFF
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h


def test_mix32_matches_integer_restatement():
    xs = [0, 1, 2, 0xFFFFFFFF, 0x9E3779B9, 123456789, 0x80000000]
    assert rck.mix32(np.array(xs, dtype=np.uint32)).tolist() == [_mix32_py(x) for x in xs]
    k = rck.policy_keys(1234, 4097, 401, np.array([0, 5, 255]), 1)
    e = (401 * 0x9E3779B9 + 4097 * 0x632BE5AB) & 0xFFFFFFFF
    want = [1234 ^ _mix32_py(e) ^ _mix32_py((i * 0x85EBCA77 + 1) & 0xFFFFFFFF) for i in (0, 5, 255)]
    assert k.tolist() == want


def test_device_sum_order():
    rng = np.random.RandomState(3)
    for n in (0, 1, 63, 64, 65, 200, 256, 257, 1000, 2048):
        r = rng.choice(np.array([-0.005, -0.105, 0.095, 4.895, -0.1, 0.1], dtype=np.float32), n)
        for lanes in (64, 256, 512):
            got = rck.device_sum(r, lanes)
            assert got.dtype == np.float32
            assert abs(float(got) - float(r.astype(np.float64).sum())) <= 1e-4 * max(1.0, n)
    # one lane per element, one wave: the butterfly tree exactly
    r = np.arange(64, dtype=np.float32) * np.float32(0.1)
    x = r.copy()
    for o in (32, 16, 8, 4, 2, 1):
        x = (x + x[np.arange(64) ^ o]).astype(np.float32)
    assert rck.device_sum(r, 64).tobytes() == x[0].tobytes()


def test_rush_restatement_without_noise_is_the_numpy_rush_policy():
    """At eps = 0 the device policy is the rush rule alone, which bd.rush_policy (the fixtures' policy)
    also implements: both agree on every agent of a fight on the oracle."""
    env, h = common.battle_env(common.ORACLE_LIB, 40)
    left, right = bd.block_positions(40, 64)
    shift = min(p[0] for p in right) - max(p[0] for p in left) - 1
    right = [[x - shift, y, d] for x, y, d in right]      # the fronts touch: rush attacks from step 0
    env.reset()
    env.add_agents(h[0], method="custom", pos=left)
    env.add_agents(h[1], method="custom", pos=right)
    base, v2a = env.get_view2attack(h[0])
    rng = np.random.RandomState(0)
    attacks = 0
    for t in range(30):
        acts = []
        for g in range(2):
            v, f = env.get_observation(h[g])
            ids = env.get_agent_id(h[g])
            a = rck.device_rush_actions(v, f, ids, g, 3, t, 99, 0.0, v2a, base, 21)
            b = bd.rush_policy(v, f, rng, v2a, base, 21, eps=0.0)
            assert a.tobytes() == b.tobytes(), (t, g)
            attacks += int((a >= base).sum())
            acts.append(a)
        for g in range(2):
            env.set_action(h[g], acts[g])
        env.step()
        env.clear_dead()
    assert attacks > 0


def test_rush_restatement_noise_rate():
    """eps of the actions come from the counter hash (about eps of them, reproducibly)."""
    ids = np.arange(4096)
    f = np.zeros((4096, 34), dtype=np.float32)
    v = np.zeros((4096, 13, 13, 7), dtype=np.float32)
    v2a = -np.ones((13, 13), dtype=np.int32)
    a = rck.device_rush_actions(v, f, ids, 0, 7, 11, 1234, 0.2, v2a, 13, 21)
    b = rck.device_rush_actions(v, f, ids, 0, 7, 11, 1234, 0.2, v2a, 13, 21)
    assert a.tobytes() == b.tobytes()
    frac = float((a != bd.MOVE_RIGHT).mean())
    assert 0.17 < frac < 0.23                     # 20 % noise, 1/21 of it lands on MOVE_RIGHT again


def test_replay_counters_and_stagger():
    """An EnvReplay of a staggered env: its first episode ends max_steps - phase steps in (or at done),
    agent-steps count the agents present at get_observation, kills count deaths."""
    left, right = bd.block_positions(64, 128)
    E, max_steps = 8, 40
    rep = rck.EnvReplay(64, [left, right], 6, E, max_steps, True, 1234, 0.2, "k_rollout")
    assert rep.ep_len == 6 * max_steps // E
    rep.advance(max_steps - rep.ep_len)
    assert rep.stats[0] == 1.0 and rep.ep_len == 0          # restarted at the cap (no side wins that fast)
    steps = max_steps - 6 * max_steps // E
    assert rep.agent_steps <= 256 * steps and (rep.agent_steps == 256 * steps) == (rep.stats[3] == 0)
    st = rep.state()
    assert [len(x) for x in st["ids"]] == [128, 128]       # the new episode's template
    assert all(np.all(x == 10.0) for x in st["hp"])
    rep.advance(rep.t + 5)
    assert rep.last["n"] == [len(x) for x in rep.last["actions"]]
