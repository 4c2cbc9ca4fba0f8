"""IsingMultiAgentEnv (reference multiagent/environment.py:49-114) without the gym dependency.

step(action_n[N, 1]) -> (obs_n, reward_n, done_n, order_param, n_up, n_down), with obs_n a list
of float64 neighbour-spin arrays and reward_n a list of float64 (1,) arrays, as the reference.
The per-agent queries go through the scenario callbacks given at construction; a missing callback
answers with the reference's defaults (empty observation, zero reward, never done)."""
import numpy as np


class Discrete:
    def __init__(self, n):
        self.n = n


class MultiBinary:
    def __init__(self, n):
        self.n = n


_DEFAULTS = {"observation": lambda: np.zeros(0), "reward": lambda: 0.0, "done": lambda: False}


class IsingMultiAgentEnv:
    metadata = {"render.modes": ["human", "rgb_array"]}

    def __init__(self, world, reset_callback=None, reward_callback=None, observation_callback=None,
                 info_callback=None, done_callback=None):
        if len(world.policy_agents) != len(world.agents):
            raise AssertionError("every Ising agent is a policy agent")
        self.world = world
        self.agents = world.policy_agents
        self.n = len(self.agents)
        self.reset_callback = reset_callback
        self.info_callback = info_callback
        self._query = {"observation": observation_callback, "reward": reward_callback, "done": done_callback}
        self.discrete_action_space = True
        self.shared_reward = False
        self.time = 0
        self.action_space = [Discrete(world.dim_spin)]
        self.observation_space = [MultiBinary(4 * world.agent_view_sight)]

    # the reference's callbacks, kept as attributes under their reference names
    reward_callback = property(lambda self: self._query["reward"])
    observation_callback = property(lambda self: self._query["observation"])
    done_callback = property(lambda self: self._query["done"])

    def _ask(self, what, agent):
        fn = self._query[what]
        return _DEFAULTS[what]() if fn is None else fn(agent, self.world)

    # gym.Env.step / reset dispatch to _step / _reset
    def step(self, action_n):
        return self._step(action_n)

    def reset(self):
        return self._reset()

    def _step(self, action_n):
        self.agents = self.world.policy_agents
        for agent, act in zip(self.agents, action_n):
            self._set_action(act, agent)
        self.world.step()
        obs_n, reward_n, done_n = [], [], []
        for a in self.agents:                     # per agent: observation, reward, done (callback order)
            for out, what in ((obs_n, "observation"), (reward_n, "reward"), (done_n, "done")):
                out.append(self._ask(what, a))
        if self.shared_reward:
            reward_n = [np.sum(reward_n)] * self.n
        w = self.world
        return obs_n, reward_n, done_n, w.order_param, w.n_up, w.n_down

    def _reset(self):
        self.reset_callback(self.world)
        self.agents = self.world.policy_agents
        return [self._ask("observation", a) for a in self.agents]

    def _get_obs(self, agent):
        return self._ask("observation", agent)

    def _get_reward(self, agent):
        return self._ask("reward", agent)

    def _get_done(self, agent):
        return self._ask("done", agent)

    def _set_action(self, action, agent):
        # spin 0 for a non-positive action, else 1; the action is one value per agent
        agent.action.a = 0 if action <= 0 else 1
        if len(action) != 1:
            raise AssertionError("action dimension error!")
