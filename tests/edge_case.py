"""Replay of tests/golden/battle_edge16.npz: custom walls, a duplicate placement that must be
skipped, a 5-on-1 fight, and the 0/0 minimap (x86 NaN bits 0xFFC00000) once a group is empty."""
import os

import numpy as np

import common


def check(lib_path):
    fx = np.load(os.path.join(common.GOLDEN, "battle_edge16.npz"))
    env, h = common.battle_env(lib_path, 16)
    env.reset()
    env.add_walls(method="custom", pos=[(5, 5), (5, 6), (5, 7), (9, 3)])
    env.add_agents(h[0], method="custom", pos=[(7, 7, 0)])
    env.add_agents(h[1], method="custom",
                   pos=[(6, 7, 0), (8, 7, 0), (7, 6, 0), (7, 8, 0), (6, 6, 0), (7, 8, 0)])
    t = 0
    while "view0_%d" % t in fx:
        for g in range(2):
            v, f = env.get_observation(h[g])
            assert v.tobytes() == fx["view%d_%d" % (g, t)].tobytes(), (t, g)
            assert f.tobytes() == fx["feat%d_%d" % (g, t)].tobytes(), (t, g)
        env.set_action(h[0], fx["act0_%d" % t].astype(np.int32))
        env.set_action(h[1], fx["act1_%d" % t].astype(np.int32))
        done = env.step()
        assert done == bool(fx["done_%d" % t])
        for g in range(2):
            assert env.get_reward(h[g]).tobytes() == fx["rew%d_%d" % (g, t)].tobytes()
        env.clear_dead()
        t += 1
    v, f = env.get_observation(h[1])
    assert v.tobytes() == fx["view1_final"].tobytes()   # bitwise, NaN payload included
    assert f.tobytes() == fx["feat1_final"].tobytes()
