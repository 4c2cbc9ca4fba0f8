"""Generate the Ising MF-Q golden fixtures from the REFERENCE scenario code (build container only).

    python tests/golden/make_ising_fixtures.py

The reference Ising scenario (examples/ising_model/Ising.py: _calc_mask, reset_world, reward,
observation) and world (multiagent/core.py: IsingWorld.step) are imported from /root/reference
and used as they are.  Two thin layers cannot be imported and are restated here:
  * IsingMultiAgentEnv._step/_reset (multiagent/environment.py:49-88) -- the module imports
    `gym`, which is absent from this image; its glue is three loops;
  * the tabular MF-Q loop of main_MFQ_Ising.py:84-159 -- a script with argparse at import.
Output: tests/golden/ising_*.npz (numeric arrays only) + ising_manifest.json.
"""
import importlib.util
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def load_scenario():
    sys.path.insert(0, REF)
    spec = importlib.util.spec_from_file_location("ref_ising_scenario", os.path.join(REF, "examples/ising_model/Ising.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.Scenario()


class Env:
    """environment.py:_reset/_step restated (the gym base class only dispatches to these)."""

    def __init__(self, sc, world):
        self.sc, self.world = sc, world
        self.agents = world.agents
        self.n = len(world.agents)

    def reset(self):
        self.sc.reset_world(self.world)
        return [self.sc.observation(a, self.world) for a in self.agents]

    def step(self, action_n):
        for i, a in enumerate(self.agents):
            a.action.a = 0 if action_n[i] <= 0 else 1
        self.world.step()
        obs, rew, done = [], [], []
        for a in self.agents:
            obs.append(self.sc.observation(a, self.world))
            rew.append(self.sc.reward(a, self.world))
            done.append(self.sc.done(a, self.world))
        return obs, rew, done, self.world.order_param, self.world.n_up, self.world.n_down


def run(n_agents, temperature, steps, lr=0.1, act_rate=1.0, decay_rate=0.99, decay_gap=2000, seed=13,
        q_every=50):
    """main_MFQ_Ising.py:11-159 with one episode and `steps` time steps (argument defaults kept)."""
    np.random.seed(seed)
    sc = load_scenario()
    world = sc.make_world(num_agents=n_agents, agent_view=1)
    env = Env(sc, world)
    n_states, n_actions = 4, 2
    obs = np.stack(env.reset())
    spins0 = np.array([a.state.spin for a in world.agents], dtype=np.int8)
    Q = np.zeros((n_agents, 5, n_actions))
    current_t = 0.3
    max_order, done_ = 0.0, 0
    rec = {"actions": [], "order": [], "n_up": [], "reward_sum": [], "spins": [], "q_steps": [], "q": []}
    reward_target = np.array([[2, -2], [1, -1], [0, 0], [-1, 1], [-2, 2]])
    stop = steps
    for t in range(steps):
        action = np.zeros(n_agents, dtype=np.int32)
        if t % decay_gap == 0:
            current_t *= decay_rate
        if current_t < temperature:
            current_t = temperature
        for i in range(n_agents):
            s = np.count_nonzero(obs[i] == 1)
            vals = [np.exp(Q[i, s, k] / current_t) for k in range(n_actions)]
            denom = 0
            for v in vals:
                denom += v
            action[i] = np.random.choice(n_actions, 1, p=[v / denom for v in vals])[0]
        obs_, reward, done, order_param, ups, downs = env.step(np.expand_dims(action, axis=1))
        obs_ = np.stack(obs_)
        mse = 0
        act_group = np.random.choice(n_agents, int(act_rate * n_agents), replace=False)
        for i in act_group:
            s = np.count_nonzero(obs[i] == 1)
            Q[i, s, action[i]] = Q[i, s, action[i]] + lr * (reward[i][0] - Q[i, s, action[i]])
            mse += np.power((Q[i, s, action[i]] - reward_target[s, action[i]]), 2)
        obs = obs_
        rec["actions"].append(action.astype(np.int8))
        rec["order"].append(order_param)
        rec["n_up"].append(ups)
        rec["reward_sum"].append(float(np.sum(reward)))
        rec["spins"].append(np.array([a.state.spin for a in world.agents], dtype=np.int8))
        if (t + 1) % q_every == 0:
            rec["q_steps"].append(t)
            rec["q"].append(Q.copy())
        if order_param > max_order:
            max_order = order_param
        if abs(max_order - order_param) < 0.001:
            done_ += 1
        else:
            done_ = 0
        if done_ == 500 or t > steps:
            stop = t + 1
            break
    out = {"spins0": spins0, "actions": np.stack(rec["actions"]), "order": np.array(rec["order"]),
           "n_up": np.array(rec["n_up"], dtype=np.int32), "reward_sum": np.array(rec["reward_sum"]),
           "spins": np.stack(rec["spins"]), "q_steps": np.array(rec["q_steps"], dtype=np.int32),
           "q": np.stack(rec["q"]) if rec["q"] else np.zeros((0, n_agents, 5, 2)), "q_final": Q,
           "obs_final": obs.astype(np.int8)}
    return out, stop


def run_episodes(n_agents, temperature, steps, episodes, lr=0.1, act_rate=1.0, decay_rate=0.99, decay_gap=2000,
                 seed=13):
    """main_MFQ_Ising.py:11-159 with -epi episodes: for i_episode: env.reset(), Q := 0, current_t := 0.3,
    the step loop until its own early stop; one np.random stream over the whole run."""
    np.random.seed(seed)
    sc = load_scenario()
    world = sc.make_world(num_agents=n_agents, agent_view=1)
    env = Env(sc, world)
    n_actions = 2
    out = {}
    for ep in range(episodes):
        obs = np.stack(env.reset())
        spins0 = np.array([a.state.spin for a in world.agents], dtype=np.int8)
        max_order, done_ = 0.0, 0
        Q = np.zeros((n_agents, 5, n_actions))
        current_t = 0.3
        acts, orders, nups = [], [], []
        stop = steps
        for t in range(steps):
            action = np.zeros(n_agents, dtype=np.int32)
            if t % decay_gap == 0:
                current_t *= decay_rate
            if current_t < temperature:
                current_t = temperature
            for i in range(n_agents):
                s = np.count_nonzero(obs[i] == 1)
                vals = [np.exp(Q[i, s, k] / current_t) for k in range(n_actions)]
                denom = 0
                for v in vals:
                    denom += v
                action[i] = np.random.choice(n_actions, 1, p=[v / denom for v in vals])[0]
            obs_, reward, done, order_param, ups, downs = env.step(np.expand_dims(action, axis=1))
            obs_ = np.stack(obs_)
            act_group = np.random.choice(n_agents, int(act_rate * n_agents), replace=False)
            for i in act_group:
                s = np.count_nonzero(obs[i] == 1)
                Q[i, s, action[i]] = Q[i, s, action[i]] + lr * (reward[i][0] - Q[i, s, action[i]])
            obs = obs_
            acts.append(action.astype(np.int8))
            orders.append(order_param)
            nups.append(ups)
            if order_param > max_order:
                max_order = order_param
            if abs(max_order - order_param) < 0.001:
                done_ += 1
            else:
                done_ = 0
            if done_ == 500 or t > steps:
                stop = t + 1
                break
        p = "e%d_" % ep
        out[p + "spins0"] = spins0
        out[p + "actions"] = np.stack(acts)
        out[p + "order"] = np.array(orders)
        out[p + "n_up"] = np.array(nups, dtype=np.int32)
        out[p + "q_final"] = Q
        out[p + "stop"] = np.int32(stop)
    return out


def main():
    manifest = {"generator": "tests/golden/make_ising_fixtures.py",
                "reference": "examples/ising_model/Ising.py + multiagent/core.py (imported); "
                             "environment.py glue and main_MFQ_Ising.py loop restated (gym absent)",
                "cases": {}}
    for name, n, tau, steps in [("ising20_t08", 400, 0.8, 300), ("ising10_t05", 100, 0.5, 400),
                                ("ising20_t20", 400, 2.0, 150)]:
        out, stop = run(n, tau, steps)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        manifest["cases"][name] = {"n_agents": n, "temperature": tau, "steps": steps, "stopped_after": stop,
                                   "lr": 0.1, "act_rate": 1.0, "seed": 13, "decay_rate": 0.99, "decay_gap": 2000}
    # a run with act_rate < 1: subsets of agents updated per step (permutation draws)
    out, stop = run(100, 0.8, 200, act_rate=0.5)
    np.savez_compressed(os.path.join(HERE, "ising10_act05.npz"), **out)
    manifest["cases"]["ising10_act05"] = {"n_agents": 100, "temperature": 0.8, "steps": 200, "stopped_after": stop,
                                          "lr": 0.1, "act_rate": 0.5, "seed": 13, "decay_rate": 0.99,
                                          "decay_gap": 2000}
    # main_MFQ_Ising.py -epi 3 on a 4x4 lattice at tau 0.1: the first two episodes stop early (order
    # parameter flat for 500 steps), so each episode's draws start where the previous stop left them
    out = run_episodes(16, 0.1, 2000, 3)
    np.savez_compressed(os.path.join(HERE, "ising4_epi3.npz"), **out)
    manifest["episode_cases"] = {"ising4_epi3": {"n_agents": 16, "temperature": 0.1, "steps": 2000, "episodes": 3,
                                                 "stops": [int(out["e%d_stop" % k]) for k in range(3)], "lr": 0.1,
                                                 "act_rate": 1.0, "seed": 13, "decay_rate": 0.99, "decay_gap": 2000}}
    with open(os.path.join(HERE, "ising_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()
