"""Pursuit: 2x2 predators chase 1x1 prey (reference builtin/config/pursuit.py:6-35)."""
import magent


def get_config(map_size):
    gw = magent.gridworld
    cfg = gw.Config()
    cfg.set({"map_width": map_size, "map_height": map_size})
    chaser = cfg.register_agent_type("predator", dict(
        width=2, length=2, hp=1, speed=1, view_range=gw.CircleRange(5), attack_range=gw.CircleRange(2),
        attack_penalty=-0.2))
    runner = cfg.register_agent_type("prey", dict(
        width=1, length=1, hp=1, speed=1.5, view_range=gw.CircleRange(4), attack_range=gw.CircleRange(0)))
    predators = cfg.add_group(chaser)
    prey = cfg.add_group(runner)
    p = gw.AgentSymbol(predators, index="any")
    q = gw.AgentSymbol(prey, index="any")
    cfg.add_reward_rule(gw.Event(p, "attack", q), receiver=[p, q], value=[1, -1])
    return cfg
