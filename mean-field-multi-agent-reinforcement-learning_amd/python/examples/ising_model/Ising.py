"""Ising scenario (reference examples/ising_model/Ising.py) on the device lattice.

The spin draws are the reference's own (np.random.choice(2) per agent, in agent order), so
main_MFQ_Ising.py's seed gives the same trajectory; reward and observation are computed on the
GPU by IsingWorld.step and handed back per agent."""
import os
import sys

import numpy as np

from examples.ising_model.multiagent.core import IsingWorld, IsingAgent

_PY = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _PY not in sys.path:
    sys.path.insert(0, _PY)
from mfrl_amd.ising import IsingLattice  # noqa: E402


class Scenario:
    def make_world(self, num_agents=100, agent_view=1):
        world = IsingWorld()
        world.agent_view_sight = agent_view
        world.dim_spin = 2
        world.dim_pos = 2
        world.n_agents = num_agents
        world.shape_size = int(np.ceil(np.power(num_agents, 1.0 / world.dim_pos)))
        world.global_state = np.zeros((world.shape_size,) * world.dim_pos)
        world.field = np.zeros((world.shape_size,) * world.dim_pos)
        world.agents = [IsingAgent(view_sight=world.agent_view_sight) for _ in range(num_agents)]
        world.lattice = IsingLattice(num_agents, replicas=1, view=agent_view)
        self.reset_world(world)
        return world

    def reset_world(self, world):
        L = world.shape_size
        for i, agent in enumerate(world.agents):
            agent.name = "agent %d" % i
            agent.color = np.array([0.35, 0.35, 0.85])
            agent.state.id = i
            agent.state.p_pos = (np.array([i // L]), np.array([i % L]))
            agent.state.spin = np.random.choice(world.dim_spin)
            mask = np.zeros(world.n_agents)
            mask[world.lattice.nbr[i]] = 1
            agent.spin_mask = mask
            world.global_state[agent.state.p_pos] = agent.state.spin
        spins = world.global_state.reshape(-1).astype(np.uint8)
        world.lattice.set_spins(spins[None, :])
        world.obs = spins[world.lattice.nbr].astype(np.float64)
        n_ups = np.count_nonzero(world.global_state.flatten())
        n_downs = world.n_agents - n_ups
        world.order_param = abs(n_ups - n_downs) / (world.n_agents + 0.0)

    def reward(self, agent, world):
        return np.array([world.rewards[agent.state.id]])

    def observation(self, agent, world):
        return world.obs[agent.state.id].copy()

    def done(self, agent, world):
        return world.order_param == 1.0
