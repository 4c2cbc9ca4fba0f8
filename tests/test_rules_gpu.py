"""the reference's other builtin configs (forest, double_attack) and the
general reward DSL (RewardEngine.cc:216-443: attack / kill / collide / at / in / die / in_a_line,
and / or / not, 'any' / 'all' / fixed-index symbols, group receivers, terminal rules) on the HIP
engine, step for step against the reference build (oracle/_ref) on the same seeded scenario:
views, features, rewards, alive flags, positions, ids and done after every step."""
import os

import numpy as np
import pytest

import common

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.path.exists(common.REF_LIB), reason="oracle/_ref not built")]


def _play(lib_path, config, map_size, counts, seed, steps, walls, episodes=2):
    env, handles = common.config_env(lib_path, config, map_size)
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
            if t % 3 == 2:            # leave agents un-cleared for a while: Agent::index stays 0
                env.clear_dead()
            if done:
                break
    del env
    return out


def _compare(got, ref):
    assert len(got) == len(ref), "episode lengths differ: %d vs %d" % (len(got), len(ref))
    for t, (a, b) in enumerate(zip(got, ref)):
        for k, (x, y) in enumerate(zip(a, b)):
            assert x.shape == y.shape and x.tobytes() == y.tobytes(), "step %d field %d differs" % (t, k)


def _both(config, map_size, counts, seed, steps=40, walls=10):
    ref = _play(common.REF_LIB, config, map_size, counts, seed, steps, walls)
    got = _play(common.HIP_LIB, config, map_size, counts, seed, steps, walls)
    _compare(got, ref)
    return ref


@pytest.mark.parametrize("seed", [1, 2])
def test_forest_matches_reference(seed):
    """builtin/config/forest.py: per-group view sizes (3x3 deer, 9x9 tigers), no attack actions for
    deer, starving tigers (step_recover < 0), kill_supply > 0 (serial attack path)."""
    _both("forest", 20, (40, 30), seed)


@pytest.mark.parametrize("seed", [1, 2])
def test_double_attack_matches_reference(seed):
    """builtin/config/double_attack.py: Event(a, attack, c) & Event(b, attack, c) over two 'any' tiger
    symbols -- the DFS with `involved` marks and re-bound inferred objects."""
    ref = _both("double_attack", 14, (30, 60), seed, steps=60)
    assert any(np.any(r[8] > 0.5) for r in ref), "no double attack happened: the test is vacuous"


def _dsl_config(map_size, variant):
    import magent
    gw = magent.gridworld
    cfg = gw.Config()
    cfg.set({"map_width": map_size, "map_height": map_size, "embedding_size": 6, "minimap_mode": variant % 2 == 1})
    a_t = cfg.register_agent_type("a", dict(width=1, length=1, hp=6, speed=1, view_range=gw.CircleRange(3),
                                            attack_range=gw.CircleRange(1.5), damage=2, step_recover=0.1,
                                            attack_in_group=1, step_reward=-0.01, kill_reward=1,
                                            dead_penalty=-0.5, attack_penalty=-0.05))
    b_t = cfg.register_agent_type("b", dict(width=1, length=1, hp=4, speed=2, view_range=gw.CircleRange(3),
                                            attack_range=gw.CircleRange(1), damage=1, step_recover=-0.05,
                                            kill_supply=1, step_reward=0.01))
    g0, g1 = cfg.add_group(a_t), cfg.add_group(b_t)
    a, a2 = gw.AgentSymbol(g0, "any"), gw.AgentSymbol(g0, "any")
    b = gw.AgentSymbol(g1, "any")
    all_a, all_b = gw.AgentSymbol(g0, "all"), gw.AgentSymbol(g1, "all")
    first_a, third_b = gw.AgentSymbol(g0, 0), gw.AgentSymbol(g1, 2)
    E = gw.Event
    if variant == 0:
        cfg.add_reward_rule(E(a, "attack", b) | E(a, "kill", b), receiver=[a, b], value=[0.3, -0.2])
        cfg.add_reward_rule(E(a, "attack", a2), receiver=a2, value=-1.0)           # same-group, attack_in_group
        cfg.add_reward_rule(E(b, "collide", a) & ~E(a, "attack", b), receiver=[b, all_a], value=[0.5, 0.01])
        cfg.add_reward_rule(E(b, "die"), receiver=[b, all_b], value=[-3.0, -0.02])
        cfg.add_reward_rule(E(a, "in", ((2, 2), (map_size // 2, map_size // 2))), receiver=a, value=0.07)
        cfg.add_reward_rule(E(b, "at", (map_size // 2, map_size // 2)), receiver=b, value=9.0)
    else:
        cfg.add_reward_rule(E(first_a, "attack", b), receiver=[first_a, b], value=[2.0, -2.0])   # fixed index
        cfg.add_reward_rule(E(a, "attack", third_b), receiver=[a, third_b], value=[1.5, -1.5])   # bind index check
        cfg.add_reward_rule(E(all_a, "attack", b), receiver=all_a, value=0.25)                   # 'all' subject
        cfg.add_reward_rule(E(all_b, "in_a_line"), receiver=all_b, value=0.125)
        cfg.add_reward_rule(E(a, "kill", b) | E(b, "collide", a), receiver=[all_a, a], value=[4.0, 0.5])
        cfg.add_reward_rule(E(all_b, "die"), receiver=all_a, value=8.0, terminal=True)
        cfg.add_reward_rule(E(b, "collide", b), receiver=b, value=0.2)
    return cfg


@pytest.mark.parametrize("variant,seed", [(0, 3), (0, 4), (1, 5), (1, 6)])
def test_reward_dsl_matches_reference(variant, seed):
    _both(_dsl_config(16, variant), 16, (36, 28), seed, steps=50, walls=8)


def test_in_a_line_all_subject_small_group():
    """in_a_line on a group of <= 2 agents and a terminal rule that fires on the first step."""
    import magent
    gw = magent.gridworld
    cfg = gw.Config()
    cfg.set({"map_width": 10, "map_height": 10})
    t = cfg.register_agent_type("t", dict(width=1, length=1, hp=3, speed=1, view_range=gw.CircleRange(2),
                                          attack_range=gw.CircleRange(1), damage=1))
    g0, g1 = cfg.add_group(t), cfg.add_group(t)
    cfg.add_reward_rule(gw.Event(gw.AgentSymbol(g1, "all"), "in_a_line"), receiver=gw.AgentSymbol(g1, "all"),
                        value=1.0, terminal=True)
    _both(cfg, 10, (5, 2), 7, steps=5, walls=2)


@pytest.mark.parametrize("seed", [1, 2])
def test_pursuit_matches_reference(seed):
    """builtin/config/pursuit.py: 2x2 predators -- multi-cell placement (random and blank checks),
    moves that overlap the mover's own body, collisions (first other agent column by column),
    attacks landing on any cell of a body, removal of whole bodies, views of multi-cell agents --
    and speed-1.5 prey."""
    ref = _both("pursuit", 20, (12, 40), seed, steps=60)
    assert any(np.any(r[4] > 0.5) for r in ref), "no predator hit a prey: the test is vacuous"


def test_odd_bodies_fill_and_custom_placement():
    """2x3 and 3x1 bodies placed by 'fill' (body-size strides) and 'custom' (overlaps skipped), with
    minimap mode, starvation removing whole bodies and a kill-triggered rule."""
    import magent
    gw = magent.gridworld
    cfg = gw.Config()
    cfg.set({"map_width": 18, "map_height": 18, "minimap_mode": True, "embedding_size": 5})
    big = cfg.register_agent_type("big", dict(width=2, length=3, hp=5, speed=1, view_range=gw.CircleRange(3),
                                              attack_range=gw.CircleRange(2), damage=2, step_recover=-0.3,
                                              kill_reward=2))
    long_ = cfg.register_agent_type("long", dict(width=3, length=1, hp=3, speed=2, view_range=gw.CircleRange(2),
                                                 attack_range=gw.CircleRange(1.5), damage=1, kill_supply=1))
    g0, g1 = cfg.add_group(big), cfg.add_group(long_)
    a, b = gw.AgentSymbol(g0, "any"), gw.AgentSymbol(g1, "any")
    cfg.add_reward_rule(gw.Event(a, "kill", b) | gw.Event(b, "kill", a), receiver=[a, b], value=[1.0, 1.0])

    def run(lib_path):
        env, (h0, h1) = common.config_env(lib_path, cfg, 18)
        env.set_seed(9)
        rs = np.random.RandomState(9)
        env.reset()
        env.add_agents(h0, method="fill", pos=[2, 2], size=[7, 9])
        env.add_agents(h1, method="custom", pos=[[10, 3], [11, 3], [10, 5], [12, 8], [3, 3], [14, 12], [9, 14]])
        env.add_agents(h1, method="fill", pos=[10, 10], size=[6, 3])
        out = []
        for t in range(40):
            rec = []
            for h in (h0, h1):
                view, feat = env.get_observation(h)
                rec += [view.copy(), feat.copy()]
            for h in (h0, h1):
                env.set_action(h, rs.randint(0, env.get_action_space(h)[0], env.get_num(h)).astype(np.int32))
            done = env.step()
            for h in (h0, h1):
                rec += [env.get_reward(h).copy(), env.get_alive(h).copy(), env.get_pos(h).copy()]
            rec.append(np.array([done]))
            out.append(rec)
            env.clear_dead()
            if done:
                break
        del env
        return out

    _compare(run(common.HIP_LIB), run(common.REF_LIB))


def _mode_config(map_size, turn, food, minimap, goal=False, big=False):
    import magent
    gw = magent.gridworld
    cfg = gw.Config()
    cfg.set({"map_width": map_size, "map_height": map_size, "turn_mode": turn, "food_mode": food,
             "minimap_mode": minimap, "goal_mode": goal, "embedding_size": 6})
    hunter = cfg.register_agent_type("hunter", dict(
        width=2 if big else 1, length=3 if big else 1, hp=6, speed=1.5, view_range=gw.CircleRange(3),
        attack_range=gw.CircleRange(1.5), damage=2, step_recover=0.1, eat_ability=1.5, food_supply=2.5,
        kill_reward=3, attack_penalty=-0.1, step_reward=-0.01))
    prey = cfg.register_agent_type("prey", dict(
        width=1, length=1, hp=4, speed=1, view_range=gw.SectorRange(3, 120), attack_range=gw.CircleRange(1),
        damage=1, step_recover=-0.02, eat_ability=0.4, food_supply=1.2, kill_supply=1.0, dead_penalty=-1))
    g0, g1 = cfg.add_group(hunter), cfg.add_group(prey)
    a, b = gw.AgentSymbol(g0, "any"), gw.AgentSymbol(g1, "any")
    cfg.add_reward_rule(gw.Event(a, "attack", b), receiver=[a, b], value=[0.2, -0.2])
    cfg.add_reward_rule(gw.Event(b, "collide", a), receiver=b, value=0.05)
    return cfg


@pytest.mark.parametrize("turn,food,minimap,big,seed", [
    (True, False, False, False, 11), (True, False, True, True, 12), (False, True, True, False, 13),
    (False, True, False, True, 14), (True, True, True, False, 15), (True, True, False, True, 16)])
def test_turn_and_food_modes_match_reference(turn, food, minimap, big, seed):
    """turn_mode (random directions from the LCG, turn actions with the reference's wise = 2a - 1,
    direction-relative moves / attacks / views, bodies pivoting about their real corner) and
    food_mode (a kill leaves food_supply on the hit cell, attacks eat min(eat_ability, food), food
    blocks moves and shows on channel 1), alone and together, 1x1 and 2x3 bodies."""
    _both(_mode_config(16, turn, food, minimap, big=big), 16, (14, 30), seed, steps=60, walls=6)


def test_goal_mode_and_set_goal_rng():
    """goal_mode adds two (always zero) features; set_goal('random') draws two LCG numbers per agent
    (GridWorld.cc:729-740), which later random placements see."""
    def run(lib_path):
        env, (h0, h1) = common.config_env(lib_path, _mode_config(14, False, False, True, goal=True), 14)
        env.set_seed(21)
        env.reset()
        env.add_agents(h0, method="random", n=6)
        env._lib.gridworld_set_goal(env.game, 0, b"random", None)
        env.add_agents(h1, method="random", n=9)
        view, feat = env.get_observation(h1)
        return [feat.copy(), view.copy(), env.get_pos(h0).copy(), env.get_pos(h1).copy()]
    _compare([run(common.HIP_LIB)], [run(common.REF_LIB)])



def test_three_level_rule_matches_reference():
    """A reward rule of three DFS levels (three 'any' tigers hitting one deer: the workgroup DSL hands such rules to
    one lane's DFS) beside a two-level one (tested binding by binding across the workgroup), against the reference
    build."""
    import magent
    gw = magent.gridworld
    cfg = gw.Config()
    cfg.set({"map_width": 16, "map_height": 16, "embedding_size": 6})
    deer = cfg.register_agent_type("deer", dict(width=1, length=1, hp=5, speed=1, view_range=gw.CircleRange(1),
                                                attack_range=gw.CircleRange(0), step_recover=0.2, kill_supply=8))
    tiger = cfg.register_agent_type("tiger", dict(width=1, length=1, hp=10, speed=1, view_range=gw.CircleRange(3),
                                                  attack_range=gw.CircleRange(1), damage=1, step_recover=-0.2))
    gd, gt = cfg.add_group(deer), cfg.add_group(tiger)
    a, b, c = gw.AgentSymbol(gt, "any"), gw.AgentSymbol(gt, "any"), gw.AgentSymbol(gt, "any")
    d = gw.AgentSymbol(gd, "any")
    E = gw.Event
    cfg.add_reward_rule(E(a, "attack", d) & E(b, "attack", d) & E(c, "attack", d), receiver=[a, b, c],
                        value=[0.5, 0.25, 0.125])
    cfg.add_reward_rule(E(a, "attack", d) & E(b, "attack", d), receiver=[a, b], value=[1, 1])
    ref = _both(cfg, 16, (40, 45), 17, steps=30, walls=4)
    assert any(np.any(r[8] > 0.1) for r in ref), "no tiger was rewarded: the test is vacuous"


def test_kill_supply_over_64_attackers_matches_reference():
    """builtin/config/forest.py crowded: ~90 tiger attacks a step, past the wave form -- with kill_supply the attack
    walks the serial order there while the moves keep the parallel forms (par_step stays on)."""
    _both("forest", 24, (60, 150), 5, steps=30, walls=6)
