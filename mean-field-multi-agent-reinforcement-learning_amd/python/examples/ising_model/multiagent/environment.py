"""IsingMultiAgentEnv (reference multiagent/environment.py) without the gym dependency.

step(action_n[N, 1]) -> (obs_n, reward_n, done_n, order_param, n_up, n_down), with obs_n a list
of float64 neighbour-spin arrays and reward_n a list of float64 (1,) arrays, as the reference."""
import numpy as np


class Discrete:
    def __init__(self, n):
        self.n = n


class MultiBinary:
    def __init__(self, n):
        self.n = n


class IsingMultiAgentEnv:
    metadata = {"render.modes": ["human", "rgb_array"]}

    def __init__(self, world, reset_callback=None, reward_callback=None, observation_callback=None,
                 info_callback=None, done_callback=None):
        self.world = world
        self.agents = self.world.policy_agents
        self.n = len(world.policy_agents)
        assert self.n == len(world.agents)
        self.reset_callback = reset_callback
        self.reward_callback = reward_callback
        self.observation_callback = observation_callback
        self.info_callback = info_callback
        self.done_callback = done_callback
        self.discrete_action_space = True
        self.shared_reward = False
        self.time = 0
        self.action_space = [Discrete(self.world.dim_spin)]
        self.observation_space = [MultiBinary(4 * self.world.agent_view_sight)]

    # gym.Env.step / reset dispatch to _step / _reset
    def step(self, action_n):
        return self._step(action_n)

    def reset(self):
        return self._reset()

    def _step(self, action_n):
        self.agents = self.world.policy_agents
        for i, agent in enumerate(self.agents):
            self._set_action(action_n[i], agent)
        self.world.step()
        obs_n, reward_n, done_n = [], [], []
        for agent in self.agents:
            obs_n.append(self._get_obs(agent))
            reward_n.append(self._get_reward(agent))
            done_n.append(self._get_done(agent))
        if self.shared_reward:
            reward_n = [np.sum(reward_n)] * self.n
        return obs_n, reward_n, done_n, self.world.order_param, self.world.n_up, self.world.n_down

    def _reset(self):
        self.reset_callback(self.world)
        self.agents = self.world.policy_agents
        return [self._get_obs(agent) for agent in self.agents]

    def _get_obs(self, agent):
        if self.observation_callback is None:
            return np.zeros(0)
        return self.observation_callback(agent, self.world)

    def _get_done(self, agent):
        if self.done_callback is None:
            return False
        return self.done_callback(agent, self.world)

    def _get_reward(self, agent):
        if self.reward_callback is None:
            return 0.0
        return self.reward_callback(agent, self.world)

    def _set_action(self, action, agent):
        agent.action.a = 0 if action <= 0 else 1
        assert len(action) == 1, "action dimenion error!"
