"""HIP Battle engine parity on the GPU box (calls through the C ABI of libmagent.so).

* replays of the reference-recorded golden fixtures (bit-exact: obs bytes, ids, rewards,
  alive, positions, counts, done -- every step);
* randomized scenarios against the C oracle (same seeds, same actions), incl. walls,
  'random' placement (engine LCG), uneven groups and multi-episode LCG persistence;
* the batched device API (E envs) against E independent oracle envs.
"""
import os

import numpy as np
import pytest

import battle_driver as bd
import common

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fast", ["1", "0"])
@pytest.mark.parametrize("name", ["battle40_seq", "battle40_s1", "battle40_s2", "battle64"])
def test_hip_replays_reference_fixture(name, fast, monkeypatch):
    """fast 1: the drop-in's one-launch step (k_dropin_step, deferred set_action / clear_dead);
    0: the per-call path."""
    monkeypatch.setenv("MFX_DROPIN_FAST", fast)
    assert common.replay_case(common.HIP_LIB, name) == []


@pytest.mark.parametrize("name", ["battle256", "battle256_seq"])
def test_hip_replays_reference_large_map(name):
    """256x256 / 4096 agents through the per-call ABI (k_step_big: band-sorted moves, attack_big):
    the 60-step opening, and two full 400-step episodes in one env (late-game band order on the
    thinned map, the LCG carried across the restart)."""
    assert common.replay_case(common.HIP_LIB, name) == []


def test_hip_full_observation_tensors():
    fx = np.load(os.path.join(common.GOLDEN, "battle64.npz"))
    case = common.manifest()["cases"]["battle64"]
    env, handles = common.battle_env(common.HIP_LIB, 64)
    env.reset()
    for g, pos in common.placement_for(case, case["episodes"][0]):
        env.add_agents(handles[g], method="custom", pos=pos)
    for g in range(2):
        v, f = env.get_observation(handles[g])
        np.testing.assert_array_equal(v, fx["e0_view_s0_g%d" % g])
        np.testing.assert_array_equal(f, fx["e0_feat_s0_g%d" % g])


def test_hip_edge_case_walls_duplicates_nan_minimap():
    import edge_case
    edge_case.check(common.HIP_LIB)


def _random_scenario(lib_path, map_size, n0, n1, seed, steps, n_walls, episodes=1):
    env, h = common.battle_env(lib_path, map_size)
    env.set_seed(seed)
    rs = np.random.RandomState(seed)
    out = []
    for ep in range(episodes):
        env.reset()
        env.add_walls(method="random", n=n_walls)
        cells = rs.choice((map_size - 2) ** 2, size=n0 + n1 + 4, replace=False)
        xs, ys = 1 + cells % (map_size - 2), 1 + cells // (map_size - 2)
        pos = np.stack([xs, ys, np.zeros_like(xs)], 1)
        env.add_agents(h[0], method="custom", pos=pos[:n0].tolist() + pos[:2].tolist())   # dup -> skipped
        env.add_agents(h[1], method="random", n=n1)
        _, v2a = env.get_view2attack(h[0])
        prs = np.random.RandomState(seed + 1000 * ep)
        for t in range(steps):
            obs = [env.get_observation(h[g]) for g in range(2)]
            rec = [o[0].tobytes() + o[1].tobytes() for o in obs]
            acts = [bd.rush_policy(obs[g][0], obs[g][1], prs, v2a, 13, 21, eps=0.4) for g in range(2)]
            for g in range(2):
                env.set_action(h[g], acts[g])
            done = env.step()
            for g in range(2):
                rec.append(env.get_reward(h[g]).tobytes() + env.get_alive(h[g]).tobytes() +
                           env.get_pos(h[g]).tobytes() + env.get_agent_id(h[g]).tobytes())
            rec.append(bytes([done]))
            out.append(bd.sha(np.frombuffer(b"".join(rec), np.uint8)))
            env.clear_dead()
            if done:
                break
    del env
    return out


_SCENARIOS = [(12, 5, 9, 1, 6), (20, 30, 30, 2, 20), (33, 60, 40, 3, 50), (64, 128, 128, 4, 0), (110, 300, 250, 5, 100)]
# envs too large for k_step's LDS copy: k_step_big (attack_big, band sort, move_jump) on random crowds -- one run each:
# these maps never take the drop-in's fast step, so MFX_DROPIN_FAST=0 would repeat the same path
_LARGE = [(180, 1500, 1500, 6, 300), (256, 2500, 2000, 7, 600)]


@pytest.mark.parametrize("map_size,n0,n1,seed,walls,fast",
                         [s + (f,) for s in _SCENARIOS for f in ("1", "0")] + [s + ("1",) for s in _LARGE])
def test_hip_matches_oracle_random_scenarios(map_size, n0, n1, seed, walls, fast, monkeypatch):
    monkeypatch.setenv("MFX_DROPIN_FAST", fast)
    ref = _random_scenario(common.ORACLE_LIB, map_size, n0, n1, seed, 60, walls, episodes=2)
    got = _random_scenario(common.HIP_LIB, map_size, n0, n1, seed, 60, walls, episodes=2)
    assert len(got) == len(ref)
    first_bad = next((i for i, (a, b) in enumerate(zip(got, ref)) if a != b), None)
    assert first_bad is None, "first divergence at step %s" % first_bad


def test_get_info_extras_match_reference():
    """get_info extras: global_minimap, mean_info, walls_info,
    render_window_info, groups_info -- HIP engine against the reference build (oracle/_ref) on the
    same scenario (custom walls, a few steps, dead agents still listed before clear_dead)."""
    if not os.path.exists(common.REF_LIB):
        pytest.skip("reference build absent")
    import magent
    outs = {}
    for name, path in (("hip", common.HIP_LIB), ("ref", common.REF_LIB)):
        env, h = common.battle_env(path, 30)
        env.reset()
        env.add_agents(-1, method="custom", pos=[[5, 5], [5, 6], [6, 6], [20, 3]])
        left, right = bd.block_positions(30, 18)
        env.add_agents(h[0], method="custom", pos=left)
        env.add_agents(h[1], method="custom", pos=right)
        rs = np.random.RandomState(4)
        for t in range(6):
            for g in range(2):
                env.get_observation(h[g])
                env.set_action(h[g], rs.randint(0, 21, env.get_num(h[g])).astype(np.int32))
            env.step()
            if t < 5:
                env.clear_dead()
        o = {"minimap": env.get_global_minimap(7, 9).copy(), "minimap13": env.get_global_minimap(13, 13).copy(),
             "walls": env._get_walls_info().copy(), "groups": env._get_groups_info().copy()}
        for g in range(2):
            o["mean%d" % g] = env.get_mean_info(h[g]).copy()
        ai, ev = env._get_render_info((3, 25), (2, 20))
        o["render"] = sorted(ai.items())
        o["events"] = ev.shape[0]
        outs[name] = o
    for k in outs["ref"]:
        a, b = outs["hip"][k], outs["ref"][k]
        if isinstance(b, np.ndarray):
            assert a.tobytes() == b.tobytes(), k
        else:
            assert a == b, k


def test_render_frames_match_reference(tmp_path):
    """The render frame writer (RenderGenerator.cc): config.json and the
    video_<n>.txt frames (walls, agents with hp %, attack events in shuffle order) byte for byte
    against the reference build, over two episodes (a reset starts a new file)."""
    if not os.path.exists(common.REF_LIB):
        pytest.skip("reference build absent")
    counts = {}
    for name, path in (("hip", common.HIP_LIB), ("ref", common.REF_LIB)):
        d = tmp_path / name
        env, h = common.battle_env(path, 26)
        env.set_render_dir(str(d))
        rs = np.random.RandomState(11)
        counts[name] = []
        for ep in range(2):
            env.reset()
            env.add_agents(-1, method="custom", pos=[[4, 4], [4, 5]])
            left, right = bd.block_positions(26, 18)
            env.add_agents(h[0], method="custom", pos=left)
            env.add_agents(h[1], method="custom", pos=right)
            env.render()
            for t in range(7):
                for g in range(2):
                    env.get_observation(h[g])
                    env.set_action(h[g], rs.randint(0, 21, env.get_num(h[g])).astype(np.int32))
                env.step()
                env.render()
                _, ev = env._get_render_info((0, 25), (0, 25))
                counts[name].append(ev.tolist())
                env.clear_dead()
    files = sorted(p.name for p in (tmp_path / "ref").iterdir())
    assert files == sorted(p.name for p in (tmp_path / "hip").iterdir())
    assert "config.json" in files and len(files) >= 3
    for f in files:
        assert (tmp_path / "hip" / f).read_bytes() == (tmp_path / "ref" / f).read_bytes(), f
    assert counts["hip"] == counts["ref"]
    assert any(len(c) for c in counts["ref"])


def _odd_sequence(lib_path, seed):
    """Call orders around the drop-in's deferred set_action / clear_dead: observation and getters
    between step and clear_dead, a step without clear_dead, one group acting, set_action twice before
    a step, get_info extras, a reset with a clear_dead pending.  Returns the SHA of every output."""
    env, h = common.battle_env(lib_path, 24)
    rs = np.random.RandomState(seed)
    out = []

    def rec(*arrs):
        out.append(bd.sha(np.frombuffer(b"".join(np.ascontiguousarray(a).tobytes() for a in arrs), np.uint8)))

    def obs():
        for g in range(2):
            v, f = env.get_observation(h[g])
            rec(v, f, env.get_agent_id(h[g]))

    def act(g):
        n = env.get_num(h[g])
        a = rs.randint(0, 21, size=n).astype(np.int32)
        env.set_action(h[g], a)

    def getters():
        for g in range(2):
            rec(env.get_reward(h[g]), env.get_alive(h[g]), env.get_pos(h[g]), env.get_agent_id(h[g]),
                np.array([env.get_num(h[g])]))

    left, right = bd.block_positions(24, 24)
    for ep in range(2):
        env.reset()
        env.add_agents(h[0], method="custom", pos=left)
        env.add_agents(h[1], method="custom", pos=right)
        for t in range(40):
            k = t % 8
            obs()
            if k == 3:
                act(0)                                   # group 1 does not act this step
            elif k == 5:
                act(0); act(1); act(1)                   # group 1 sets its actions twice
            else:
                act(0); act(1)
            rec(np.array([env.step()]))
            getters()
            if k == 2:
                obs()                                    # before clear_dead: dead agents still listed
            if k == 4:
                rec(np.asarray(env._get_walls_info()), env.get_mean_info(h[0]), env.get_global_minimap(8, 8))
                continue                                 # no clear_dead this step
            if k == 6:
                getters()
            env.clear_dead()
            if k == 7:
                getters()
            if ep == 0 and t == 25:
                break                                    # reset with a clear_dead pending
    del env
    return out


@pytest.mark.parametrize("fast", ["1", "0"])
@pytest.mark.parametrize("seed", [1, 2])
def test_dropin_odd_call_orders(seed, fast, monkeypatch):
    """Against the reference engine itself (oracle/_ref): the extras are not in the C oracle."""
    if not os.path.exists(common.REF_LIB):
        pytest.skip("oracle/_ref not built")
    monkeypatch.setenv("MFX_DROPIN_FAST", fast)
    ref = _odd_sequence(common.REF_LIB, seed)
    got = _odd_sequence(common.HIP_LIB, seed)
    assert len(got) == len(ref)
    first_bad = next((i for i, (a, b) in enumerate(zip(got, ref)) if a != b), None)
    assert first_bad is None, "first divergence at record %s" % first_bad


@pytest.mark.parametrize("mode", ["resident_idle_exits", "one_launch_per_step", "actions_in_mailbox_poll"])
def test_dropin_resident_server_modes(mode, monkeypatch):
    """The resident drop-in server (one k_dropin_step launch answering env.step() through a mailbox)
    with an idle timeout of 20 us, so that it leaves between nearly every pair of steps and is
    relaunched with the request already posted (the relaunch race); the one-launch-per-step form
    (MFX_DROPIN_RESIDENT=0); and the tagged actions read inside the request poll (MFX_DROPIN_MAIL=1).
    All against the C oracle, two episodes with walls and random placement."""
    monkeypatch.setenv("MFX_DROPIN_FAST", "1")
    if mode == "resident_idle_exits":
        monkeypatch.setenv("MFX_DROPIN_IDLE_US", "20")
    elif mode == "one_launch_per_step":
        monkeypatch.setenv("MFX_DROPIN_RESIDENT", "0")
    else:
        monkeypatch.setenv("MFX_DROPIN_MAIL", "1")
    ref = _random_scenario(common.ORACLE_LIB, 33, 60, 40, 3, 60, 50, episodes=2)
    got = _random_scenario(common.HIP_LIB, 33, 60, 40, 3, 60, 50, episodes=2)
    assert len(got) == len(ref)
    first_bad = next((i for i, (a, b) in enumerate(zip(got, ref)) if a != b), None)
    assert first_bad is None, "first divergence at step %s" % first_bad


def test_dropin_two_resident_envs_interleaved(monkeypatch):
    """Two drop-in envs in one process, stepped alternately: two resident servers on their own streams
    at once, each answering only its own mailbox.  Each env's record stream equals the oracle's."""
    monkeypatch.setenv("MFX_DROPIN_FAST", "1")

    def run(lib, interleave):
        envs = []
        for k, (size, n) in enumerate([(24, 40), (40, 64)]):
            env, h = common.battle_env(lib, size)
            env.reset()
            left, right = bd.block_positions(size, n)
            env.add_agents(h[0], method="custom", pos=left)
            env.add_agents(h[1], method="custom", pos=right)
            _, v2a = env.get_view2attack(h[0])
            envs.append([env, h, v2a, np.random.RandomState(10 + k), [], False])
        order = [0, 1] * 40 if interleave else [0] * 40 + [1] * 40
        for k in order:
            env, h, v2a, rs, out, finished = envs[k]
            if finished:
                continue
            obs = [env.get_observation(h[g]) for g in range(2)]
            rec = [o[0].tobytes() + o[1].tobytes() for o in obs]
            for g in range(2):
                env.set_action(h[g], bd.rush_policy(obs[g][0], obs[g][1], rs, v2a, 13, 21, eps=0.3))
            done = env.step()
            for g in range(2):
                rec.append(env.get_reward(h[g]).tobytes() + env.get_alive(h[g]).tobytes())
            out.append(bd.sha(np.frombuffer(b"".join(rec) + bytes([done]), np.uint8)))
            env.clear_dead()
            envs[k][5] = done
        return [e[4] for e in envs]

    assert run(common.HIP_LIB, True) == run(common.ORACLE_LIB, False)
