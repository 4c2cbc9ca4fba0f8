"""Double attack: a tiger is paid only when another tiger hits the same deer in the same step
(reference builtin/config/double_attack.py:6-43)."""
import magent


def get_config(map_size):
    gw = magent.gridworld
    cfg = gw.Config()
    cfg.set({"map_width": map_size, "map_height": map_size, "embedding_size": 10})
    prey = cfg.register_agent_type("deer", dict(
        width=1, length=1, hp=5, speed=1, view_range=gw.CircleRange(1), attack_range=gw.CircleRange(0),
        step_recover=0.2, kill_supply=8))
    hunter = cfg.register_agent_type("tiger", dict(
        width=1, length=1, hp=10, speed=1, view_range=gw.CircleRange(4), attack_range=gw.CircleRange(1),
        damage=1, step_recover=-0.2))
    deer = cfg.add_group(prey)
    tigers = cfg.add_group(hunter)
    t1 = gw.AgentSymbol(tigers, index="any")
    t2 = gw.AgentSymbol(tigers, index="any")
    target = gw.AgentSymbol(deer, index="any")
    both = gw.Event(t1, "attack", target) & gw.Event(t2, "attack", target)
    cfg.add_reward_rule(both, receiver=[t1, t2], value=[1, 1])
    return cfg
