"""The Battle game: two armies of identical 'small' agents (reference builtin/config/battle.py:6-44)."""
import magent

SMALL_AGENT = dict(
    width=1, length=1, hp=10, speed=2,
    damage=2, step_recover=0.1,
    step_reward=-0.005, kill_reward=5, dead_penalty=-0.1, attack_penalty=-0.1,
)


def get_config(map_size):
    gw = magent.gridworld
    cfg = gw.Config()
    cfg.set({"map_width": map_size, "map_height": map_size, "minimap_mode": True, "embedding_size": 10})
    attrs = dict(SMALL_AGENT)
    attrs["view_range"] = gw.CircleRange(6)
    attrs["attack_range"] = gw.CircleRange(1.5)
    small = cfg.register_agent_type("small", attrs)
    armies = [cfg.add_group(small), cfg.add_group(small)]
    a, b = (gw.AgentSymbol(g, index="any") for g in armies)
    # shaping: +0.2 for every (non-lethal) hit on the other army
    cfg.add_reward_rule(gw.Event(a, "attack", b), receiver=a, value=0.2)
    cfg.add_reward_rule(gw.Event(b, "attack", a), receiver=b, value=0.2)
    return cfg
