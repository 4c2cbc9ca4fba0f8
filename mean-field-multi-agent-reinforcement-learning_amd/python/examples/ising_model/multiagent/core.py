"""Ising world whose spins live on the GPU (reference multiagent/core.py).

IsingWorld.step() sets every agent's spin to its action on the device lattice and brings back
what the scenario callbacks read: rewards, neighbour observations, n_up/n_down, order parameter.
"""
import numpy as np


class IsingEntityState:
    def __init__(self):
        self.id = None
        self.p_pos = None


class IsingAgentState(IsingEntityState):
    def __init__(self):
        super().__init__()
        self.spin = None


class IsingAction:
    def __init__(self):
        self.a = None


class IsingEntity:
    def __init__(self):
        self.name = ""
        self.size = 0.050
        self.movable = False
        self.color = None
        self.state = IsingEntityState()


class IsingAgent(IsingEntity):
    def __init__(self, view_sight=1):
        super().__init__()
        self.movable = False
        self.view_sight = view_sight
        self.spin_mask = None
        self.state = IsingAgentState()
        self.state.spin_range = [0, 1]
        self.action = IsingAction()
        self.action.a_range = [0, 1]
        self.action_callback = None


class IsingWorld:
    def __init__(self):
        self.agents = []
        self.n_agents = 1
        self.agent_view_sight = 1
        self.dim_pos = 2
        self.dim_spin = 2
        self.dim_color = 3
        self.shape_size = 1
        self.global_state = None
        self.moment = 1
        self.field = None
        self.temperature = .1
        self.interaction = 1
        self.order_param = 1.0
        self.order_param_delta = 0.01
        self.n_up = 0
        self.n_down = 0
        # device side (set by Scenario.make_world)
        self.lattice = None
        self.rewards = None          # float64 [N] of the last step
        self.obs = None              # float64 [N, K] neighbour spins

    @property
    def entities(self):
        return self.agents

    @property
    def policy_agents(self):
        return [a for a in self.agents if a.action_callback is None]

    @property
    def scripted_agents(self):
        return [a for a in self.agents if a.action_callback is not None]

    def step(self):
        for agent in self.scripted_agents:
            agent.action = agent.action_callback(agent, self)
        actions = np.array([0 if a.action.a == 0 else 1 for a in self.agents], dtype=np.int32)
        rew, obs, n_up, order = self.lattice.step(actions[None, :])
        self.rewards = rew[0]
        self.obs = obs[0].astype(np.float64)
        flat = self.global_state.reshape(-1)
        flat[:] = actions
        for a, s in zip(self.agents, actions):
            a.state.spin = int(s)
        self.n_up = int(n_up[0])
        self.n_down = self.n_agents - self.n_up
        self.order_param = float(order[0])
