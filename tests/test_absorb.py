"""can_absorb agent types (AgentType.h:40; Map::do_move's absorption, Map.cc:345-364; the minimap and
move filters, GridWorld.cc:357-363 / :638; render_window_info and the frame writer, GridWorld.cc:905-906,
RenderGenerator.cc:129-160).  A mover that walks into an agent of a can_absorb type that is not absorbed
yet dies and leaves the map; the occupant is marked absorbed, its hp doubles and it stops moving.  When
the OBSERVING group's type can absorb, absorbed agents leave every group's minimap density and its
divisor (the reference tests agents[0] of the observed group).

Parity against the reference build (oracle/_ref) on the same seeded scenarios: the C oracle on the CPU,
the HIP engine on the GPU (views, features, rewards, alive flags, positions, ids, done after every step;
render_window_info and the render frames).  No reference config ships a can_absorb type, so the
scenarios are synthetic (two groups, random walls, random actions)."""
import os

import numpy as np
import pytest

import common

needs_ref = pytest.mark.skipif(not os.path.exists(common.REF_LIB), reason="oracle/_ref not built")


def absorb_config(map_size, minimap, absorber_views):
    """Group 0 hunters (speed 2, they die by walking into blobs), group 1 blobs (can_absorb).
    absorber_views: the blobs also see (their view range matters for the minimap quirk)."""
    import magent
    gw = magent.gridworld
    cfg = gw.Config()
    cfg.set({"map_width": map_size, "map_height": map_size, "embedding_size": 5, "minimap_mode": minimap})
    hunter = cfg.register_agent_type("hunter", dict(width=1, length=1, hp=5, speed=2, view_range=gw.CircleRange(3),
                                                    attack_range=gw.CircleRange(1), damage=1, step_recover=0.1,
                                                    step_reward=-0.01, kill_reward=1, dead_penalty=-0.5,
                                                    attack_penalty=-0.02))
    blob = cfg.register_agent_type("blob", dict(width=1, length=1, hp=3, speed=1, can_absorb=True,
                                                view_range=gw.CircleRange(absorber_views),
                                                attack_range=gw.CircleRange(1), damage=1, step_recover=0.0,
                                                step_reward=0.01))
    g0, g1 = cfg.add_group(hunter), cfg.add_group(blob)
    a, b = gw.AgentSymbol(g0, "any"), gw.AgentSymbol(g1, "any")
    cfg.add_reward_rule(gw.Event(a, "collide", b), receiver=[a, b], value=[-1.0, 2.0])
    cfg.add_reward_rule(gw.Event(a, "attack", b), receiver=a, value=0.3)
    return cfg


def play(lib_path, cfg, map_size, counts, seed, steps, walls, episodes=2, probe=None):
    """Per step: views / features of both groups, then rewards, alive, positions, ids, done.  probe (a
    list): absorbed blobs per step, from render_window_info (the reference build / HIP engine only)."""
    env, handles = common.config_env(lib_path, cfg, map_size)
    env.set_seed(seed)
    rs = np.random.RandomState(seed)
    out = []
    for ep in range(episodes):
        env.reset()
        env.add_walls(method="random", n=walls)
        for h, n in zip(handles, counts):
            env.add_agents(h, method="random", n=n)
        for t in range(steps):
            rec = []
            for h in handles:
                view, feat = env.get_observation(h)
                rec += [view.copy(), feat.copy()]
            for h in handles:
                n_act = env.get_action_space(h)[0]
                env.set_action(h, rs.randint(0, n_act, env.get_num(h)).astype(np.int32))
            done = env.step()
            for h in handles:
                rec += [env.get_reward(h).copy(), env.get_alive(h).copy(), env.get_pos(h).copy(),
                        env.get_agent_id(h).copy()]
            rec.append(np.array([done]))
            out.append(rec)
            if probe is not None:
                ai, _ = env._get_render_info((0, map_size), (0, map_size))
                probe.append(sum(1 for v in ai.values() if v[2] == 1))
            if t % 2 == 1:
                env.clear_dead()
            if done:
                break
    del env
    return out


def compare(got, ref):
    assert len(got) == len(ref), "episode lengths differ: %d vs %d" % (len(got), len(ref))
    for t, (a, b) in enumerate(zip(got, ref)):
        for k, (x, y) in enumerate(zip(a, b)):
            assert x.shape == y.shape and x.tobytes() == y.tobytes(), "step %d field %d differs" % (t, k)


CASES = [(True, 2, 1), (False, 3, 2), (True, 4, 3)]     # minimap, blob view radius, seed


@needs_ref
@pytest.mark.parametrize("minimap,view,seed", CASES)
def test_oracle_absorb_matches_reference(minimap, view, seed):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    absorbed = []
    ref = play(common.REF_LIB, absorb_config(16, minimap, view), 16, (40, 30), seed, 40, 6, probe=absorbed)
    got = play(common.ORACLE_LIB, absorb_config(16, minimap, view), 16, (40, 30), seed, 40, 6)
    compare(got, ref)
    assert max(absorbed) >= 3, "too few blobs absorbed: the scenario is vacuous (%s)" % absorbed


@pytest.mark.gpu
@needs_ref
@pytest.mark.parametrize("minimap,view,seed", CASES)
def test_hip_absorb_matches_reference(minimap, view, seed):
    pr, pg = [], []
    ref = play(common.REF_LIB, absorb_config(16, minimap, view), 16, (40, 30), seed, 40, 6, probe=pr)
    got = play(common.HIP_LIB, absorb_config(16, minimap, view), 16, (40, 30), seed, 40, 6, probe=pg)
    compare(got, ref)
    assert pg == pr and max(pr) >= 3


@pytest.mark.gpu
@needs_ref
def test_hip_absorb_render_matches_reference(tmp_path):
    """render_window_info lists only absorbed blobs; the frame writer draws and counts only them."""
    outs = {}
    for name, path in (("hip", common.HIP_LIB), ("ref", common.REF_LIB)):
        d = tmp_path / name
        env, h = common.config_env(path, absorb_config(14, True, 2), 14)
        env.set_render_dir(str(d))
        env.set_seed(9)
        rs = np.random.RandomState(9)
        env.reset()
        env.add_agents(h[0], method="random", n=40)
        env.add_agents(h[1], method="random", n=30)
        info = []
        for t in range(12):
            for g in range(2):
                env.get_observation(h[g])
                env.set_action(h[g], rs.randint(0, env.get_action_space(h[g])[0], env.get_num(h[g])).astype(np.int32))
            env.step()
            env.render()
            ai, ev = env._get_render_info((0, 13), (0, 13))
            info.append((sorted(ai.items()), ev.shape[0]))
            env.clear_dead()
        outs[name] = info
    assert outs["hip"] == outs["ref"]
    assert any(len(i[0]) for i in outs["ref"]), "no blob was absorbed: the test is vacuous"
    files = sorted(p.name for p in (tmp_path / "ref").iterdir())
    assert files == sorted(p.name for p in (tmp_path / "hip").iterdir())
    for f in files:
        assert (tmp_path / "hip" / f).read_bytes() == (tmp_path / "ref" / f).read_bytes(), f
