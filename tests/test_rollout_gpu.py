"""The fused rollout kernel (k_rollout, bench path) against the C oracle.

Every env of the batch is replayed on the oracle with the actions the on-device policy
chose; observations (views + features), rewards, mean actions (former_act_prob) and the
episode restart at max_steps must match bit for bit."""
import os

import numpy as np
import pytest

import battle_driver as bd
import common
import rollout_check as rck

pytestmark = pytest.mark.gpu


def _run(map_size, n_side, E, T, max_steps, config="battle", VF=13 * 13 * 7, F=34, path=None):
    import torch
    from mfrl_amd.battle import BattleBatch
    left, right = bd.block_positions(map_size, n_side)
    eng = BattleBatch(map_size, E, config=config, stream=torch.cuda.current_stream())
    eng.rollout_init([left, right], max_steps=max_steps, eps=0.3, seed=99, stagger=False)
    if path is not None:
        assert eng.rollout_path() == path, eng.rollout_path()
    rc = eng.rowcap
    NA = eng.env.get_action_space(eng.handles[0])[0]
    recs = []
    for t in range(T):
        eng.rollout_step(1)
        r = {}
        for g in range(2):
            r["view%d" % g] = torch.empty(E * rc * VF, dtype=torch.float32)
            r["feat%d" % g] = torch.empty(E * rc * F, dtype=torch.float32)
            eng.rollout_copy("view", r["view%d" % g], group=g)
            eng.rollout_copy("feature", r["feat%d" % g], group=g)
        r["act"] = torch.empty(E * 2 * rc, dtype=torch.int32)
        r["rew"] = torch.empty(E * 2 * rc, dtype=torch.float32)
        r["mean"] = torch.empty(E * 2 * NA, dtype=torch.float64)
        eng.rollout_copy("actions", r["act"])
        eng.rollout_copy("rewards", r["rew"])
        eng.rollout_copy("mean_action", r["mean"])
        eng.sync()
        recs.append({k: v.numpy() for k, v in r.items()})
    return recs, rc


PATHS = {"fused": ("0", "0", "k_rollout"), "pipe": ("1", "0", "k_rollout_obs+k_rollout"),
         "queue": ("0", None, "k_rollout_bigq")}


@pytest.mark.parametrize("path", sorted(PATHS))
@pytest.mark.parametrize("map_size,n_side,E,T,max_steps", [(24, 18, 3, 45, 20), (64, 128, 2, 70, 400)])
def test_rollout_matches_oracle(map_size, n_side, E, T, max_steps, path, monkeypatch):
    """fused: k_rollout; pipe: k_rollout_obs beside k_rollout<.., kSplit> (two state copies); queue: the
    queue kernel k_rollout_bigq, which takes batches of few LDS-sized envs by default (small_e_max)."""
    pipe, small_e, want = PATHS[path]
    monkeypatch.setenv("MFX_ROLLOUT_PIPE", pipe)
    if small_e is not None:
        monkeypatch.setenv("MFX_SMALL_E", small_e)
    recs, rc = _run(map_size, n_side, E, T, max_steps, path=want)
    left, right = bd.block_positions(map_size, n_side)
    VF, F = 13 * 13 * 7, 34
    for e in range(E):
        env, h = common.battle_env(common.ORACLE_LIB, map_size)
        ep_len = 0
        env.reset()
        env.add_agents(h[0], method="custom", pos=left)
        env.add_agents(h[1], method="custom", pos=right)
        for t in range(T):
            r = recs[t]
            acts = []
            for g in range(2):
                v, f = env.get_observation(h[g])
                n = len(v)
                gv = r["view%d" % g].reshape(E, rc, VF)[e, :n]
                gf = r["feat%d" % g].reshape(E, rc, F)[e, :n]
                assert gv.tobytes() == v.reshape(n, VF).tobytes(), (e, t, g, "view")
                assert gf.tobytes() == f.tobytes(), (e, t, g, "feature")
                a = r["act"].reshape(E, 2, rc)[e, g, :n].astype(np.int32)
                acts.append(a)
                mean = np.mean(list(map(lambda x: np.eye(21)[x], a)), axis=0) if n else np.zeros(21)
                assert r["mean"].reshape(E, 2, 21)[e, g].tobytes() == mean.tobytes(), (e, t, g, "mean")
            for g in range(2):
                env.set_action(h[g], acts[g])
            done = env.step()
            for g in range(2):
                rw = env.get_reward(h[g])
                assert r["rew"].reshape(E, 2, rc)[e, g, :len(rw)].tobytes() == rw.tobytes(), (e, t, g, "reward")
            env.clear_dead()
            ep_len += 1
            if done or ep_len >= max_steps:
                ep_len = 0
                env.reset()
                env.add_agents(h[0], method="custom", pos=left)
                env.add_agents(h[1], method="custom", pos=right)
        del env


@pytest.mark.parametrize("pipe", ["0", "1"])
def test_rollout_processes_every_env_once(pipe, monkeypatch):
    """The persistent work queue (the heaviest-first class lists filed by the previous launch, read
    through the per-launch counter) hands every env to exactly one workgroup per launch: before the
    armies meet no agent dies, so each env's agent-step counter must read 256 * steps.  E (5003) is
    not a multiple of the persistent grid or of the filing buffer (32 envs per flush)."""
    monkeypatch.setenv("MFX_ROLLOUT_PIPE", pipe)
    import torch
    from mfrl_amd.battle import BattleBatch
    E, steps = 5003, 3
    left, right = bd.block_positions(64, 128)
    eng = BattleBatch(64, E, stream=torch.cuda.current_stream())
    eng.rollout_init([left, right], max_steps=400, eps=0.0, seed=7, stagger=False)
    grid, lds = eng.rollout_info()
    assert 0 < grid <= E and lds > 0
    eng.rollout_step(steps)
    got = torch.empty(E, dtype=torch.int64)
    eng.rollout_copy("agent_steps", got)
    eng.sync()
    assert (got == 256 * steps).all(), np.unique(got.numpy())


@pytest.mark.parametrize("map_size,n_side,E,T,max_steps", [(256, 2048, 2, 34, 30), (200, 1250, 3, 24, 400)])
def test_rollout_large_env_matches_oracle(map_size, n_side, E, T, max_steps):
    """Envs too large for one workgroup's LDS: rollout_step runs k_observe per group and
    k_rollout_big (state in HBM, 1024-lane parallel exact step).  Checked in lockstep against one
    oracle env per batch env: views, features, actions' mean, rewards, the episode restart."""
    import torch
    from mfrl_amd.battle import BattleBatch
    left, right = bd.block_positions(map_size, n_side)
    eng = BattleBatch(map_size, E, stream=torch.cuda.current_stream())
    eng.rollout_init([left, right], max_steps=max_steps, eps=0.3, seed=5, stagger=False)
    grid, lds = eng.rollout_info()
    assert grid == E and lds > 64 * 1024          # the large-env path was chosen
    assert eng.rollout_path() == "k_rollout_bigq"
    rc = eng.rowcap
    VF, F = 13 * 13 * 7, 34
    envs = []
    for e in range(E):
        env, h = common.battle_env(common.ORACLE_LIB, map_size)
        env.reset()
        env.add_agents(h[0], method="custom", pos=left)
        env.add_agents(h[1], method="custom", pos=right)
        envs.append((env, h))
    ep_len, kills = [0] * E, 0
    for t in range(T):
        eng.rollout_step(1)
        view = [torch.empty(E * rc * VF, dtype=torch.float32) for _ in range(2)]
        feat = [torch.empty(E * rc * F, dtype=torch.float32) for _ in range(2)]
        act = torch.empty(E * 2 * rc, dtype=torch.int32)
        rew = torch.empty(E * 2 * rc, dtype=torch.float32)
        mean = torch.empty(E * 2 * 21, dtype=torch.float64)
        for g in range(2):
            eng.rollout_copy("view", view[g], group=g)
            eng.rollout_copy("feature", feat[g], group=g)
        eng.rollout_copy("actions", act)
        eng.rollout_copy("rewards", rew)
        eng.rollout_copy("mean_action", mean)
        eng.sync()
        for e, (env, h) in enumerate(envs):
            acts = []
            for g in range(2):
                v, f = env.get_observation(h[g])
                n = len(v)
                assert view[g].numpy().reshape(E, rc, VF)[e, :n].tobytes() == v.reshape(n, VF).tobytes(), (e, t, g)
                assert feat[g].numpy().reshape(E, rc, F)[e, :n].tobytes() == f.tobytes(), (e, t, g)
                a = act.numpy().reshape(E, 2, rc)[e, g, :n].astype(np.int32)
                acts.append(a)
                m = np.bincount(a, minlength=21) / n if n else np.full(21, np.nan)
                assert np.array_equal(mean.numpy().reshape(E, 2, 21)[e, g], m, equal_nan=True), (e, t, g)
            for g in range(2):
                env.set_action(h[g], acts[g])
            done = env.step()
            for g in range(2):
                rw = env.get_reward(h[g])
                kills += int((~env.get_alive(h[g])).sum())
                assert rew.numpy().reshape(E, 2, rc)[e, g, :len(rw)].tobytes() == rw.tobytes(), (e, t, g, "reward")
            env.clear_dead()
            ep_len[e] += 1
            if done or ep_len[e] >= max_steps:
                ep_len[e] = 0
                env.reset()
                env.add_agents(h[0], method="custom", pos=left)
                env.add_agents(h[1], method="custom", pos=right)
    eng.rollout_check()                           # the queue kernel never stalled
    assert kills > 0                              # the attack fixed point saw real kills


def test_rollout_pipe_state_handoff(monkeypatch):
    """The pipeline's two state copies trade places every launch: after an odd number of launches the
    per-call API must see the same state as the fused kernel leaves, and rollout steps after per-call
    calls (a re-plan) must continue identically."""
    import torch
    from mfrl_amd.battle import BattleBatch
    E, VF, F = 3, 13 * 13 * 7, 34
    left, right = bd.block_positions(64, 128)
    engs = []
    monkeypatch.setenv("MFX_SMALL_E", "0")           # k_rollout even for 3 envs
    for pipe in ("0", "1"):
        monkeypatch.setenv("MFX_ROLLOUT_PIPE", pipe)
        eng = BattleBatch(64, E, stream=torch.cuda.current_stream())
        eng.rollout_init([left, right], max_steps=400, eps=0.3, seed=3, stagger=False)
        engs.append(eng)

    def snap(eng):
        rc = eng.rowcap
        out = []
        for g in range(2):
            v = torch.zeros(E * rc * VF, dtype=torch.float32, device="cuda")
            f = torch.zeros(E * rc * F, dtype=torch.float32, device="cuda")
            eng.observe(g, v, f, rc)
            out += [v, f]
        n = torch.empty(E * 2, dtype=torch.int32, device="cuda")
        eng.rollout_copy("group_num", n)
        eng.sync()
        return [x.cpu().numpy() for x in out + [n]]

    def rollout_out(eng):
        rc = eng.rowcap
        out = []
        for g in range(2):
            v = torch.empty(E * rc * VF, dtype=torch.float32, device="cuda")
            eng.rollout_copy("view", v, group=g)
            out.append(v)
        a = torch.empty(E * 2 * rc, dtype=torch.int32, device="cuda")
        eng.rollout_copy("actions", a)
        eng.sync()
        return [x.cpu().numpy() for x in out + [a]]

    for eng in engs:
        eng.rollout_step(37)                     # odd: the pipeline's live state is its second copy
    a, b = snap(engs[0]), snap(engs[1])
    for x, y in zip(a, b):
        assert x.tobytes() == y.tobytes()
    for eng in engs:
        eng.rollout_step(4)
    for x, y in zip(rollout_out(engs[0]), rollout_out(engs[1])):
        assert x.tobytes() == y.tobytes()


def _generic_config(map_size):
    """Battle rules with an 11x11 view, no minimap and 8-bit ids: not the Battle shape, so k_rollout runs
    its generic observation path (obs_rows) and per-id minimap bins."""
    import magent
    gw = magent.gridworld
    cfg = gw.Config()
    cfg.set({"map_width": map_size, "map_height": map_size, "minimap_mode": False, "embedding_size": 8})
    attrs = dict(width=1, length=1, hp=10, speed=2, damage=2, step_recover=0.1, step_reward=-0.005,
                 kill_reward=5, dead_penalty=-0.1, attack_penalty=-0.1,
                 view_range=gw.CircleRange(5), attack_range=gw.CircleRange(1.5))
    small = cfg.register_agent_type("small", attrs)
    armies = [cfg.add_group(small), cfg.add_group(small)]
    a, b = (gw.AgentSymbol(g, index="any") for g in armies)
    cfg.add_reward_rule(gw.Event(a, "attack", b), receiver=a, value=0.2)
    cfg.add_reward_rule(gw.Event(b, "attack", a), receiver=b, value=0.2)
    return cfg


def test_rollout_generic_shape_matches_oracle():
    """k_rollout<kB = false> (a view size other than Battle's 13x13 and no minimap) against the oracle."""
    import magent
    map_size, n_side, E, T, max_steps = 32, 40, 2, 40, 30
    cfg = _generic_config(map_size)
    probe = common.config_env(common.ORACLE_LIB, cfg, map_size)[0]
    ph = probe.get_handles()
    vh, vw, nc = probe.get_view_space(ph[0])
    F = probe.get_feature_space(ph[0])[0]
    NA = probe.get_action_space(ph[0])[0]
    VF = vh * vw * nc
    assert (vh, vw) == (11, 11) and F != 34
    del probe
    recs, rc = _run(map_size, n_side, E, T, max_steps, config=cfg, VF=VF, F=F)
    left, right = bd.block_positions(map_size, n_side)
    for e in range(E):
        env, h = common.config_env(common.ORACLE_LIB, cfg, map_size)
        ep_len = 0
        env.reset()
        env.add_agents(h[0], method="custom", pos=left)
        env.add_agents(h[1], method="custom", pos=right)
        for t in range(T):
            r = recs[t]
            acts = []
            for g in range(2):
                v, f = env.get_observation(h[g])
                n = len(v)
                assert r["view%d" % g].reshape(E, rc, VF)[e, :n].tobytes() == v.reshape(n, VF).tobytes(), (e, t, g)
                assert r["feat%d" % g].reshape(E, rc, F)[e, :n].tobytes() == f.tobytes(), (e, t, g)
                acts.append(r["act"].reshape(E, 2, rc)[e, g, :n].astype(np.int32))
            for g in range(2):
                env.set_action(h[g], acts[g])
            done = env.step()
            for g in range(2):
                rw = env.get_reward(h[g])
                assert r["rew"].reshape(E, 2, rc)[e, g, :len(rw)].tobytes() == rw.tobytes(), (e, t, g, "reward")
            env.clear_dead()
            ep_len += 1
            if done or ep_len >= max_steps:
                ep_len = 0
                env.reset()
                env.add_agents(h[0], method="custom", pos=left)
                env.add_agents(h[1], method="custom", pos=right)
        del env


def _sample_envs(E, k=16):
    """k envs spread over the batch, both ends included (env E-1 has the shortest first episode)."""
    return sorted(set([0, 1, E // 2, E - 2, E - 1] + [int(x) for x in np.linspace(0, E - 1, k - 5)]))[:k]


def _check_launches(eng, map_size, n_side, envs, T, S, max_steps, seed, eps, path):
    """Run T steps as launches of S steps; after EVERY launch compare the sampled envs with their oracle
    replays (tests/rollout_check.py: last step's observation / actions / rewards / mean action, the state
    after it, agent-steps, episode statistics, running return; device and queue error words)."""
    assert eng.rollout_path() == path, eng.rollout_path()
    chk = rck.RolloutChecker(eng, map_size, bd.block_positions(map_size, n_side), envs, max_steps, True, seed, eps)
    restarts_before = [r.stats[0] for r in chk.replays]
    t = 0
    while t < T:
        k = min(S, T - t)
        eng.rollout_step(k)
        t += k
        bad = chk.check(t)
        assert not bad, bad[:8]
    assert all(r.stats[0] > b for r, b in zip(chk.replays, restarts_before))     # every sampled env restarted


def test_rollout_bench_shape_matches_oracle():
    """The 64x64 bench exactly as bench.py runs it: 131072 staggered envs (the persistent grid is far
    smaller than E, so the heaviest-first class queue, the register prefetch and the queue hand-off are
    live; view offsets past 2^31 floats), 20 steps per k_rollout launch, 456 steps (every env restarts at
    least once; the bench's preparation + warmup + timed window is 425).  16 sampled envs are replayed on
    the C oracle from rollout_init on with the host restatement of the device rush policy, and compared
    after every launch.  Stagger: env e's first episode starts at length e * max_steps // E
    (BattleEngine::rollout_init)."""
    import torch
    from mfrl_amd.battle import BattleBatch
    E, T, S, max_steps, seed = 131072, 456, 20, 400, 1234
    left, right = bd.block_positions(64, 128)
    eng = BattleBatch(64, E, stream=torch.cuda.current_stream())
    eng.rollout_init([left, right], max_steps=max_steps, eps=0.2, seed=seed, stagger=True)
    eng.rollout_substeps(S)
    grid, _ = eng.rollout_info()
    assert grid < E                                  # the work queue hands out envs
    _check_launches(eng, 64, 128, _sample_envs(E), T, S, max_steps, seed, 0.2, "k_rollout")


@pytest.mark.parametrize("E", [8, 64])
def test_rollout_small_e_matches_oracle(E):
    """configs[3]'s per-GPU shape (64 envs over 8 GPUs = 8 per GPU; and 64 on one GPU) as bench.py runs it:
    64x64 envs on the queue kernel (small_e_max), 20 steps per launch, 420 steps (every env restarts).
    Every env (E = 8) or 8 sampled envs (E = 64) replayed on the C oracle, compared after every launch."""
    import torch
    from mfrl_amd.battle import BattleBatch
    T, S, max_steps, seed = 420, 20, 400, 1234
    left, right = bd.block_positions(64, 128)
    eng = BattleBatch(64, E, stream=torch.cuda.current_stream())
    eng.rollout_init([left, right], max_steps=max_steps, eps=0.2, seed=seed, stagger=True)
    eng.rollout_substeps(S)
    _check_launches(eng, 64, 128, rck.sample_envs(E, 8), T, S, max_steps, seed, 0.2, "k_rollout_bigq")


def test_rollout_bigq_bench_shape_matches_oracle():
    """The 256x256 bench (configs[4]) exactly as bench.py runs it: 2048 staggered envs of 2048 + 2048
    agents, 20 steps per k_rollout_bigq launch, 420 steps (every env restarts, most inside a launch).
    8 sampled envs replayed on the C oracle from rollout_init on, compared after every launch."""
    import torch
    from mfrl_amd.battle import BattleBatch
    E, T, S, max_steps, seed = 2048, 420, 20, 400, 1234
    left, right = bd.block_positions(256, 2048)
    eng = BattleBatch(256, E, stream=torch.cuda.current_stream())
    eng.rollout_init([left, right], max_steps=max_steps, eps=0.2, seed=seed, stagger=True)
    eng.rollout_substeps(S)
    _check_launches(eng, 256, 2048, _sample_envs(E, 8), T, S, max_steps, seed, 0.2, "k_rollout_bigq")


@pytest.mark.parametrize("E,S", [(2048, 20), (1, 1)])
def test_rollout_bigq_matches_reference_recording(E, S):
    """k_rollout_bigq against the REFERENCE engine's own recording (tests/golden/battle256_rollout.npz,
    make_battle_fixtures.py): env 0 of the 256x256 batch (2048 + 2048 agents, device rush policy, seed
    1234) through two full 400-step episodes -- the late-game band order, clear_dead churn, the restart
    and the LCG across it.  (2048, 20): the bench's batch and launch shape, compared at every launch
    boundary; (1, 1): one env, compared after every step."""
    import torch
    from mfrl_amd.battle import BattleBatch
    fx = rck.RolloutFixture()
    c = fx.case
    assert E in (1, c["n_envs"])          # env 0 starts at episode length 0 for any batch size
    eng = BattleBatch(c["map_size"], E, stream=torch.cuda.current_stream())
    eng.rollout_init(fx.placement, max_steps=c["max_steps"], eps=c["eps"], seed=c["seed"], stagger=True)
    eng.rollout_substeps(S)
    assert eng.rollout_path() == "k_rollout_bigq", eng.rollout_path()
    assert eng.rollout_sum_lanes(65) == 512           # the recording's reward sums are in 512-lane order
    t = 0
    while t < c["steps"]:
        k = min(S, c["steps"] - t)
        eng.rollout_step(k)
        t += k
        eng.rollout_check()
        bad = fx.compare(rck.device_records(eng, [0]), 0, t - 1)
        assert not bad, bad[:8]
    assert fx.restart.sum() == 2


@pytest.mark.parametrize("E,S,path", [(131072, 20, "k_rollout"), (8, 0, "k_rollout_bigq"), (1, 1, "k_rollout_bigq")])
def test_rollout_matches_reference_recording_64(E, S, path):
    """The headline kernel against the REFERENCE engine's own recording (tests/golden/battle64_rollout.npz,
    make_battle_fixtures.py): env 0 of the 64x64 bench batch (128 + 128 agents, device rush policy,
    seed 1234) through two full 400-step episodes.  (131072, 20): k_rollout at the bench's batch and launch shape,
    compared at every launch boundary; (8, 0): configs[3]'s per-GPU batch on the pipelined few-env stepper with the
    engine's steps per launch, compared every 20 steps; (1, 1): one env, after every step.  The episode returns
    follow the engine's own reward-sum teams (rollout_sum_lanes), which the recording holds in every order."""
    import torch
    from mfrl_amd.battle import BattleBatch
    c = common.manifest()["cases"]["battle64_rollout"]
    eng = BattleBatch(c["map_size"], E, stream=torch.cuda.current_stream())
    left, right = bd.block_positions(64, 128)
    eng.rollout_init([left, right], max_steps=c["max_steps"], eps=c["eps"], seed=c["seed"], stagger=True)
    eng.rollout_substeps(S)
    assert eng.rollout_path() == path, eng.rollout_path()
    fx = rck.RolloutFixture("battle64_rollout", (eng.rollout_sum_lanes(64), eng.rollout_sum_lanes(65)))
    K = S if S > 0 else 20
    t = 0
    while t < c["steps"]:
        k = min(K, c["steps"] - t)
        eng.rollout_step(k)
        t += k
        eng.rollout_check()
        bad = fx.compare(rck.device_records(eng, [0]), 0, t - 1)
        assert not bad, bad[:8]
    assert fx.restart.sum() == 2


def test_rollout_bigq_bench_shape_matches_reference_build():
    """The 256x256 bench batch (2048 staggered envs, 20 steps per launch, 420 steps) with 4 sampled envs
    replayed on the reference engine itself (oracle/_ref, one thread) instead of the C oracle."""
    import torch
    from mfrl_amd.battle import BattleBatch
    if not os.path.exists(common.REF_LIB):
        pytest.skip("oracle/_ref not built")
    E, T, S, max_steps, seed = 2048, 420, 20, 400, 1234
    left, right = bd.block_positions(256, 2048)
    eng = BattleBatch(256, E, stream=torch.cuda.current_stream())
    eng.rollout_init([left, right], max_steps=max_steps, eps=0.2, seed=seed, stagger=True)
    eng.rollout_substeps(S)
    assert eng.rollout_path() == "k_rollout_bigq"
    chk = rck.RolloutChecker(eng, 256, [left, right], [1, 700, 1500, E - 1], max_steps, True, seed, 0.2,
                             lib=common.REF_LIB)
    t = 0
    while t < T:
        eng.rollout_step(S)
        t += S
        bad = chk.check(t)
        assert not bad, bad[:8]
    assert all(r.stats[0] >= 1 for r in chk.replays)


def test_rollout_large_env_staggered_many_envs_matches_oracle():
    """The large-env pipeline with more envs than XCD item lists: 16 staggered 200x200 envs (1250 per
    side) in two sub-batch pipelines, so each of the 8 per-XCD observation item lists holds an env
    of each sub-batch and the workgroups of every XCD help the others' lists; 32 steps with an
    episode cap of 24 (every env restarts).  Every env replayed on the C oracle: views, features,
    rewards, mean actions, bit for bit."""
    import torch
    from mfrl_amd.battle import BattleBatch
    E, T, max_steps, VF, F, M = 16, 32, 24, 13 * 13 * 7, 34, 200
    left, right = bd.block_positions(M, 1250)
    eng = BattleBatch(M, E, stream=torch.cuda.current_stream())
    eng.rollout_init([left, right], max_steps=max_steps, eps=0.3, seed=99, stagger=True)
    grid, lds = eng.rollout_info()
    assert lds > 64 * 1024                           # the large-env path
    assert eng.rollout_path() == "k_rollout_bigq"
    rc = eng.rowcap
    envs = []
    for e in range(E):
        env, h = common.battle_env(common.ORACLE_LIB, M)
        env.reset()
        env.add_agents(h[0], method="custom", pos=left)
        env.add_agents(h[1], method="custom", pos=right)
        envs.append([env, h, e * max_steps // E])
    restarts = 0
    for t in range(T):
        eng.rollout_step(1)
        view = [torch.empty(E * rc * VF, dtype=torch.float32) for _ in range(2)]
        feat = [torch.empty(E * rc * F, dtype=torch.float32) for _ in range(2)]
        act = torch.empty(E * 2 * rc, dtype=torch.int32)
        rew = torch.empty(E * 2 * rc, dtype=torch.float32)
        mean = torch.empty(E * 2 * 21, dtype=torch.float64)
        for g in range(2):
            eng.rollout_copy("view", view[g], group=g)
            eng.rollout_copy("feature", feat[g], group=g)
        eng.rollout_copy("actions", act)
        eng.rollout_copy("rewards", rew)
        eng.rollout_copy("mean_action", mean)
        eng.sync()
        for e, st in enumerate(envs):
            env, h, _ = st
            acts = []
            for g in range(2):
                v, f = env.get_observation(h[g])
                n = len(v)
                assert view[g].numpy().reshape(E, rc, VF)[e, :n].tobytes() == v.reshape(n, VF).tobytes(), (e, t, g)
                assert feat[g].numpy().reshape(E, rc, F)[e, :n].tobytes() == f.tobytes(), (e, t, g)
                a = act.numpy().reshape(E, 2, rc)[e, g, :n].astype(np.int32)
                acts.append(a)
                m = np.bincount(a, minlength=21) / n if n else np.full(21, np.nan)
                assert np.array_equal(mean.numpy().reshape(E, 2, 21)[e, g], m, equal_nan=True), (e, t, g)
            for g in range(2):
                env.set_action(h[g], acts[g])
            done = env.step()
            for g in range(2):
                rw = env.get_reward(h[g])
                assert rew.numpy().reshape(E, 2, rc)[e, g, :len(rw)].tobytes() == rw.tobytes(), (e, t, g, "reward")
            env.clear_dead()
            st[2] += 1
            if done or st[2] >= max_steps:
                st[2] = 0
                restarts += 1
                env.reset()
                env.add_agents(h[0], method="custom", pos=left)
                env.add_agents(h[1], method="custom", pos=right)
    eng.rollout_check()
    assert restarts >= E


def test_rollout_large_env_renumbered_slots_per_call():
    """Large envs renumber their slots to the list order at every rollout clear_dead
    (clear_dead_renumber): after kills a slot is no longer the agent's id, which lives on in rid, and the
    reference's id_counter runs ahead of the slots in use (rid_off).  Per-call calls on that state must
    still answer as the reference does: get_agent_id (batched getter and the drop-in's env-0 record),
    add_agents (new agents take the reference's next ids), a per-call observation (features embed the id),
    a per-call step with attacks and clear_dead -- and rollout launches after them (a re-seed) continue
    the oracle replay bit for bit."""
    import torch
    from mfrl_amd.battle import BattleBatch, GET_HP, GET_ID, GET_POS, GET_REWARD
    E, M, n_side, T, T2, seed, eps = 2, 200, 1250, 24, 12, 5, 0.3
    placement = bd.block_positions(M, n_side)
    eng = BattleBatch(M, E, stream=torch.cuda.current_stream())
    eng.rollout_init(placement, max_steps=400, eps=eps, seed=seed, stagger=False)
    assert eng.rollout_path() == "k_rollout_bigq"
    chk = rck.RolloutChecker(eng, M, placement, list(range(E)), 400, False, seed, eps)
    eng.rollout_step(T)
    bad = chk.check(T)
    assert not bad, bad[:8]
    reps = chk.replays
    assert all(sum(rep.oracle.get_num(h) for h in rep.h) < 2 * n_side for rep in reps)   # kills: renumbered
    rc, VF, F = eng.rowcap, 13 * 13 * 7, 34
    H = eng.handles

    def per_group(what, dt, w=1):
        out = []
        for g in range(2):
            buf = torch.empty((E, rc, w), dtype=dt, device="cuda")
            eng.get(g, what, buf, rc)
            out.append(buf)
        eng.sync()
        return [x.cpu().numpy() for x in out]

    def compare_state(tag):
        ids, pos, hp = per_group(GET_ID, torch.int32), per_group(GET_POS, torch.int32, 2), per_group(GET_HP, torch.float32)
        for e, rep in enumerate(reps):
            for g in range(2):
                want = rep.oracle.get_agent_id(rep.h[g])
                m = len(want)
                assert ids[g][e, :m, 0].tobytes() == want.tobytes(), (tag, e, g, "ids")
                assert pos[g][e, :m].tobytes() == rep.oracle.get_pos(rep.h[g]).tobytes(), (tag, e, g, "pos")
                got_hp = rep.oracle._info_array(rep.h[g], b"hp", (m,), np.float32)
                assert hp[g][e, :m, 0].tobytes() == got_hp.tobytes(), (tag, e, g, "hp")
        for g in range(2):      # the drop-in's env-0 record (k_get_env0)
            assert eng.env.get_agent_id(H[g]).tobytes() == reps[0].oracle.get_agent_id(reps[0].h[g]).tobytes(), (tag, g)

    compare_state("after the rollout")
    eng.env.add_agents(H[0], method="random", n=7)
    for rep in reps:
        rep.oracle.add_agents(rep.h[0], method="random", n=7)
    compare_state("after add_agents")
    assert int(reps[0].oracle.get_agent_id(reps[0].h[0])[-1]) == 2 * n_side + 6      # the reference's next ids
    view = [torch.empty(E * rc * VF, dtype=torch.float32, device="cuda") for _ in range(2)]
    feat = [torch.empty(E * rc * F, dtype=torch.float32, device="cuda") for _ in range(2)]
    for g in range(2):
        eng.observe(g, view[g], feat[g], rc)
    eng.sync()
    rng = np.random.RandomState(3)
    acts = torch.zeros((2, E, rc), dtype=torch.int32)
    for e, rep in enumerate(reps):
        for g in range(2):
            v, f = rep.oracle.get_observation(rep.h[g])
            n = len(v)
            assert view[g].cpu().numpy().reshape(E, rc, VF)[e, :n].tobytes() == v.reshape(n, VF).tobytes(), (e, g)
            assert feat[g].cpu().numpy().reshape(E, rc, F)[e, :n].tobytes() == f.tobytes(), (e, g)
            a = rng.randint(0, 21, size=n).astype(np.int32)
            acts[g, e, :n] = torch.from_numpy(a)
            rep.oracle.set_action(rep.h[g], a)
    for g in range(2):
        eng.set_action(g, acts[g].cuda().contiguous(), rc)
    eng.step()
    for rep in reps:
        rep.oracle.step()
    rew = per_group(GET_REWARD, torch.float32)
    for e, rep in enumerate(reps):
        for g in range(2):
            rw = rep.oracle.get_reward(rep.h[g])
            assert rew[g][e, :len(rw), 0].tobytes() == rw.tobytes(), (e, g, "reward")
    eng.clear_dead()
    for rep in reps:
        rep.oracle.clear_dead()
    compare_state("after a per-call step")
    eng.rollout_step(T2)                             # re-seed; the replays continue on the changed oracles
    bad = chk.check(T + T2)
    assert not bad, bad[:8]


def test_rollout_large_env_queue_matches_pipeline(monkeypatch):
    """The queue-driven large-env kernel (k_rollout_bigq: observation items and the steps they gate in
    one launch, several steps of every env per launch, items filed inside the launch) against the
    two-stream pipeline (k_observe_items + k_rollout_big, checked on the oracle above): 24 staggered
    200x200 envs, episode cap 24 (restarts inside launches), 1 and 5 steps per launch; every output
    buffer bit for bit after 13 and 43 steps, and no stalled queue."""
    import ctypes
    import torch
    from mfrl_amd.battle import BattleBatch
    E, M = 24, 200
    left, right = bd.block_positions(M, 1250)
    engs = []
    for fused, sub in (("0", 1), ("1", 1), ("1", 5)):
        monkeypatch.setenv("MFX_BIG_FUSED", fused)
        eng = BattleBatch(M, E, stream=torch.cuda.current_stream())
        eng.rollout_init([left, right], max_steps=24, eps=0.3, seed=41, stagger=True)
        eng.rollout_substeps(sub)
        assert eng.rollout_path() == ("k_rollout_bigq" if fused == "1" else "k_observe_items+k_rollout_big")
        engs.append(eng)

    N = 1250                 # rows every env wrote at its first step (the rows past them were never written)

    def dump(eng):
        out, rc = [], eng.rowcap
        for name, dt in (("actions", torch.int32), ("rewards", torch.float32), ("mean_action", torch.float64),
                         ("stats", torch.float64), ("agent_steps", torch.int64), ("group_num", torch.int32),
                         ("episode_return", torch.float32)):
            ptr, nb = ctypes.c_void_p(), ctypes.c_size_t()
            eng._dll.mfx_battle_rollout_buffer(eng.game, name.encode(), 0, ctypes.byref(ptr), ctypes.byref(nb))
            x = torch.empty(nb.value // torch.tensor([], dtype=dt).element_size(), dtype=dt, device="cuda")
            eng.rollout_copy(name, x)
            out.append(x.view(E, 2, rc)[:, :, :N].contiguous() if name in ("actions", "rewards") else x)
        for g in range(2):
            for name, w in (("view", 13 * 13 * 7), ("feature", 34)):
                x = torch.empty(E * rc * w, dtype=torch.float32, device="cuda")
                eng.rollout_copy(name, x, group=g)
                out.append(x.view(E, rc, w)[:, :N].contiguous())
        return out

    for n in (13, 30):
        for eng in engs:
            eng.rollout_step(n)
        for eng in engs:
            eng.rollout_check()
        ref = dump(engs[0])
        for j, other in enumerate(engs[1:]):
            got = dump(other)
            torch.cuda.synchronize()
            for k, (x, y) in enumerate(zip(ref, got)):
                if not torch.equal(x.view(torch.uint8), y.view(torch.uint8)):
                    bad = (x.view(torch.uint8) != y.view(torch.uint8)).view(x.shape[0], x.shape[1], -1).any(-1)
                    idx = bad.nonzero()[:12].tolist()
                    gn = ref[5].view(E, 2).tolist()
                    raise AssertionError((n, k, j, idx, [gn[i[0]] for i in idx], int(bad.sum())))
            del got
        del ref


def test_rollout_bigq_reseed_after_per_call_ops(monkeypatch):
    """Per-call calls between queue-kernel launches: after an even number of launches the
    last launch's filings for the next launch sit unconsumed in parity 0 under the live tag; per-call
    steps with attacks and clear_dead shrink the groups, so the re-seed files fewer items than those
    slots hold.  The re-seed must clear them (or k_rollout_bigq would take stale words for items).
    32-agent items (MFX_BIGQ_ROWS), so a few deaths change the filing counts.  Checked against the
    two-stream pipeline given the same per-call calls: every output buffer, the statistics and counters
    bit for bit, and no queue error."""
    import ctypes
    import torch
    from mfrl_amd.battle import BattleBatch
    E, M, S, R = 24, 200, 5, 32
    left, right = bd.block_positions(M, 1250)
    monkeypatch.setenv("MFX_BIGQ_ROWS", str(R))
    engs = []
    for fused in ("0", "1"):
        monkeypatch.setenv("MFX_BIG_FUSED", fused)
        eng = BattleBatch(M, E, stream=torch.cuda.current_stream())
        eng.rollout_init([left, right], max_steps=60, eps=0.3, seed=17, stagger=True)
        eng.rollout_substeps(S)
        engs.append(eng)
    assert engs[1].rollout_path() == "k_rollout_bigq"
    rc = engs[0].rowcap

    def dump(eng):
        out = []
        for name, dt in (("actions", torch.int32), ("rewards", torch.float32), ("mean_action", torch.float64),
                         ("stats", torch.float64), ("agent_steps", torch.int64), ("group_num", torch.int32),
                         ("episode_return", torch.float32)):
            ptr, nb = ctypes.c_void_p(), ctypes.c_size_t()
            eng._dll.mfx_battle_rollout_buffer(eng.game, name.encode(), 0, ctypes.byref(ptr), ctypes.byref(nb))
            x = torch.empty(nb.value // torch.tensor([], dtype=dt).element_size(), dtype=dt, device="cuda")
            eng.rollout_copy(name, x)
            # (rows past those every env wrote at its first step hold allocation garbage)
            out.append(x.view(E, 2, rc)[:, :, :1250].contiguous() if name in ("actions", "rewards") else x)
        for g in range(2):
            for name, w in (("view", 13 * 13 * 7), ("feature", 34)):
                x = torch.empty(E * rc * w, dtype=torch.float32, device="cuda")
                eng.rollout_copy(name, x, group=g)
                out.append(x.view(E, rc, w)[:, :1250].contiguous())
        return out

    sizes = []
    for eng in engs:
        eng.rollout_step(2 * S)                      # two launches: the stale filings are in parity 0
        eng.rollout_check()
        n0 = torch.empty(E * 2, dtype=torch.int32, device="cuda")
        eng.rollout_copy("group_num", n0)
        acts = torch.empty(E * 2 * rc, dtype=torch.int32, device="cuda")
        for _ in range(6):                           # per-call steps: the last step's actions again
            eng.rollout_copy("actions", acts)
            for g in range(2):
                eng.set_action(g, acts.view(E, 2, rc)[:, g].contiguous(), rc)
            eng.step()
            eng.clear_dead()
        n1 = torch.empty(E * 2, dtype=torch.int32, device="cuda")
        eng.rollout_copy("group_num", n1)
        eng.sync()
        items = [int(((n + R - 1) // R).sum().item()) for n in (n0, n1)]
        sizes.append((n0.sum().item(), n1.sum().item(), items[0], items[1]))
        eng.rollout_step(13)                         # re-seed, then 3 launches
        eng.rollout_check()
    assert sizes[0] == sizes[1] and sizes[0][3] < sizes[0][2], sizes       # fewer items to file
    a, b = dump(engs[0]), dump(engs[1])
    torch.cuda.synchronize()
    for k, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x.view(torch.uint8), y.view(torch.uint8)), k


def test_rollout_bigq_bench_shape_matches_pipeline(monkeypatch):
    """The 256x256 bench's own shape (configs[4]: 2048 staggered envs of 2048 + 2048 agents, episode cap
    400, 20 steps per k_rollout_bigq launch) against the two-stream pipeline at one step per launch,
    after 420 steps (every env restarts at least once, inside a launch for most): every output
    buffer bit for bit (all rows the first step wrote), the episode statistics, the agent-step
    counters, and no stalled queue."""
    import ctypes
    import torch
    from mfrl_amd.battle import BattleBatch
    E, M, N, T = 2048, 256, 2048, 420
    left, right = bd.block_positions(M, N)
    engs = []
    for fused, sub in (("0", 1), ("1", 20)):
        monkeypatch.setenv("MFX_BIG_FUSED", fused)
        eng = BattleBatch(M, E, stream=torch.cuda.current_stream())
        eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=1234, stagger=True)
        eng.rollout_substeps(sub)
        assert eng.rollout_path() == ("k_rollout_bigq" if fused == "1" else "k_observe_items+k_rollout_big")
        eng.rollout_step(T)
        engs.append(eng)
    engs[1].rollout_check()
    rc = engs[0].rowcap
    for name, dt in (("actions", torch.int32), ("rewards", torch.float32), ("mean_action", torch.float64),
                     ("stats", torch.float64), ("agent_steps", torch.int64), ("group_num", torch.int32),
                     ("episode_return", torch.float32)):
        xs = []
        for eng in engs:
            ptr, nb = ctypes.c_void_p(), ctypes.c_size_t()
            eng._dll.mfx_battle_rollout_buffer(eng.game, name.encode(), 0, ctypes.byref(ptr), ctypes.byref(nb))
            x = torch.empty(nb.value // torch.tensor([], dtype=dt).element_size(), dtype=dt, device="cuda")
            eng.rollout_copy(name, x)
            xs.append(x.view(E, 2, rc)[:, :, :N] if name in ("actions", "rewards") else x)
        torch.cuda.synchronize()
        assert torch.equal(xs[0].view(torch.uint8) if xs[0].is_contiguous() else xs[0].contiguous().view(torch.uint8),
                           xs[1].view(torch.uint8) if xs[1].is_contiguous() else xs[1].contiguous().view(torch.uint8)), name
    for g in range(2):
        for name, w in (("feature", 34), ("view", 13 * 13 * 7)):
            xs = []
            for eng in engs:
                x = torch.empty(E * rc * w, dtype=torch.float32, device="cuda")
                eng.rollout_copy(name, x, group=g)
                xs.append(x.view(E, rc, w)[:, :N])
            torch.cuda.synchronize()
            same = torch.equal(xs[0].view(torch.int32), xs[1].view(torch.int32))
            assert same, (name, g, int((xs[0].view(torch.int32) != xs[1].view(torch.int32)).any(-1).sum()))
            del xs


@pytest.mark.parametrize("sub", [2, 7, 20, 64])
def test_rollout_substeps_match_single_steps(sub):
    """k_rollout running `sub` consecutive steps of each env per launch (image kept in LDS) leaves
    exactly what single-step launches leave: every output buffer, the episode statistics, the
    agent-step counters and the state the per-call API observes, after a partial episode and again
    after a full episode cap (restarts inside a launch).  Together with the oracle replay above this
    pins the multi-step launch."""
    import torch
    from mfrl_amd.battle import BattleBatch
    E = 3000
    left, right = bd.block_positions(64, 128)
    engs = []
    for s in (1, sub):
        eng = BattleBatch(64, E, stream=torch.cuda.current_stream())
        eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=77, stagger=True)
        eng.rollout_substeps(s)
        engs.append(eng)

    def dump(eng):
        out = []
        for name, dt in (("actions", torch.int32), ("rewards", torch.float32), ("mean_action", torch.float64),
                         ("stats", torch.float64), ("agent_steps", torch.int64), ("group_num", torch.int32),
                         ("episode_return", torch.float32)):
            import ctypes
            ptr, nb = ctypes.c_void_p(), ctypes.c_size_t()
            eng._dll.mfx_battle_rollout_buffer(eng.game, name.encode(), 0, ctypes.byref(ptr), ctypes.byref(nb))
            x = torch.empty(nb.value // torch.tensor([], dtype=dt).element_size(), dtype=dt, device="cuda")
            eng.rollout_copy(name, x)
            out.append(x)
        for g in range(2):
            for name, w in (("view", 13 * 13 * 7), ("feature", 34)):
                x = torch.empty(E * eng.rowcap * w, dtype=torch.float32, device="cuda")
                eng.rollout_copy(name, x, group=g)
                out.append(x)
        return out

    for n in (37, 400):
        for eng in engs:
            eng.rollout_step(n)
        a, b = dump(engs[0]), dump(engs[1])
        torch.cuda.synchronize()
        for k, (x, y) in enumerate(zip(a, b)):
            assert torch.equal(x.view(torch.uint8) if x.dtype != torch.uint8 else x,
                               y.view(torch.uint8) if y.dtype != torch.uint8 else y), (n, k)
        del a, b
    # and the per-call API sees the same state (cells rebuilt from the fused rollout's image)
    rc = engs[0].rowcap
    snaps = []
    for eng in engs:
        v = torch.zeros(E * rc * 13 * 13 * 7, dtype=torch.float32, device="cuda")
        f = torch.zeros(E * rc * 34, dtype=torch.float32, device="cuda")
        eng.observe(1, v, f, rc)
        eng.sync()
        snaps.append((v, f))
    assert torch.equal(snaps[0][0], snaps[1][0]) and torch.equal(snaps[0][1], snaps[1][1])


def _mixed_action_config(map_size):
    """Battle rules where group 1 attacks only its 4 orthogonal neighbours: n_action 21 and 17, so the
    [E][G][21] mean-action rows hold 17 entries for group 1 (stride = the largest n_action)."""
    import magent
    gw = magent.gridworld
    cfg = gw.Config()
    cfg.set({"map_width": map_size, "map_height": map_size, "minimap_mode": True, "embedding_size": 10})
    base = dict(width=1, length=1, hp=10, speed=2, view_range=gw.CircleRange(6), damage=2, step_recover=0.1,
                step_reward=-0.005, kill_reward=5, dead_penalty=-0.1, attack_penalty=-0.1)
    t0 = cfg.register_agent_type("wide", dict(base, attack_range=gw.CircleRange(1.5)))
    t1 = cfg.register_agent_type("cross", dict(base, attack_range=gw.CircleRange(1)))
    armies = [cfg.add_group(t0), cfg.add_group(t1)]
    a, b = (gw.AgentSymbol(g, index="any") for g in armies)
    cfg.add_reward_rule(gw.Event(a, "attack", b), receiver=a, value=0.2)
    cfg.add_reward_rule(gw.Event(b, "attack", a), receiver=b, value=0.2)
    return cfg


def test_rollout_mixed_n_action_mean_rows():
    """Groups with different n_action: every group's mean action lands in its own row of the
    [E][G][max n_action] buffer (no overlap between groups or envs), checked against the oracle."""
    import torch
    from mfrl_amd.battle import BattleBatch
    map_size, n_side, E, T = 32, 40, 3, 30
    cfg = _mixed_action_config(map_size)
    probe = common.config_env(common.ORACLE_LIB, cfg, map_size)[0]
    ph = probe.get_handles()
    nas = [probe.get_action_space(h)[0] for h in ph]
    assert nas == [21, 17], nas
    del probe
    left, right = bd.block_positions(map_size, n_side)
    eng = BattleBatch(map_size, E, config=cfg, stream=torch.cuda.current_stream())
    eng.rollout_init([left, right], max_steps=400, eps=0.3, seed=4, stagger=False)
    rc, NA = eng.rowcap, 21
    oracles = []
    for e in range(E):
        env, h = common.config_env(common.ORACLE_LIB, cfg, map_size)
        env.reset()
        env.add_agents(h[0], method="custom", pos=left)
        env.add_agents(h[1], method="custom", pos=right)
        oracles.append((env, h))
    for t in range(T):
        eng.rollout_step(1)
        act = torch.empty(E * 2 * rc, dtype=torch.int32)
        mean = torch.full((E * 2 * NA,), -7.0, dtype=torch.float64)
        eng.rollout_copy("actions", act)
        eng.rollout_copy("mean_action", mean)
        eng.sync()
        for e, (env, h) in enumerate(oracles):
            acts = []
            for g in range(2):
                n = len(env.get_observation(h[g])[0])
                a = act.numpy().reshape(E, 2, rc)[e, g, :n].astype(np.int32)
                acts.append(a)
                want = np.bincount(a, minlength=nas[g]) / n if n else np.full(nas[g], np.nan)
                row = mean.numpy().reshape(E, 2, NA)[e, g]
                assert np.array_equal(row[:nas[g]], want, equal_nan=True), (e, t, g)
            for g in range(2):
                env.set_action(h[g], acts[g])
            done = env.step()
            env.clear_dead()
            if done:
                env.reset()
                env.add_agents(h[0], method="custom", pos=left)
                env.add_agents(h[1], method="custom", pos=right)


def _dump_rollout(eng, E, N):
    """Every rollout output buffer of a batch (rows < N, the rows every env wrote at its first step) and the
    per-call getters' ids / positions / hp, as uint8 tensors on the device."""
    import ctypes
    import torch
    from mfrl_amd.battle import GET_HP, GET_ID, GET_POS
    rc, out = eng.rowcap, []
    for name, dt in (("actions", torch.int32), ("rewards", torch.float32), ("mean_action", torch.float64),
                     ("stats", torch.float64), ("agent_steps", torch.int64), ("group_num", torch.int32),
                     ("episode_return", torch.float32)):
        ptr, nb = ctypes.c_void_p(), ctypes.c_size_t()
        eng._dll.mfx_battle_rollout_buffer(eng.game, name.encode(), 0, ctypes.byref(ptr), ctypes.byref(nb))
        x = torch.empty(nb.value // torch.tensor([], dtype=dt).element_size(), dtype=dt, device="cuda")
        eng.rollout_copy(name, x)
        out.append((name, (x.view(E, 2, rc)[:, :, :N] if name in ("actions", "rewards") else x).contiguous()))
    for g in range(2):
        for name, w in (("view", 13 * 13 * 7), ("feature", 34)):
            x = torch.empty(E * rc * w, dtype=torch.float32, device="cuda")
            eng.rollout_copy(name, x, group=g)
            out.append(("%s%d" % (name, g), x.view(E, rc, w)[:, :N].contiguous()))
    n = torch.empty(E * 2, dtype=torch.int32, device="cuda")
    eng.rollout_copy("group_num", n)
    torch.cuda.synchronize()
    for what, w, dt in ((GET_ID, 1, torch.int32), (GET_POS, 2, torch.int32), (GET_HP, 1, torch.float32)):
        for g in range(2):
            buf = torch.zeros((E, rc, w), dtype=dt, device="cuda")
            eng.get(g, what, buf, rc)
            eng.sync()
            live = torch.arange(rc, device="cuda")[None, :] < n.view(E, 2)[:, g:g + 1]
            out.append(("get%d_%d" % (what, g), torch.where(live[:, :, None], buf, torch.zeros_like(buf))))
    return [(k, v.view(torch.uint8)) for k, v in out]


def test_rollout_renumber_modes_agree(monkeypatch):
    """The large-env slot renumbering changes where each agent's state sits, never a result: 24 staggered
    200x200 envs (episode cap 24: restarts inside launches), 16 steps per k_rollout_bigq launch, 64 steps, with
    the renumbering off (MFX_RENUMBER=0), on with its identity fast path (1, the default) and rewriting every
    slot at every clear_dead (2): every output buffer and the per-call ids / positions / hp bit for bit."""
    import torch
    from mfrl_amd.battle import BattleBatch
    E, M, N, T = 24, 200, 1250, 64
    left, right = bd.block_positions(M, N)
    dumps = []
    for mode in ("0", "1", "2"):
        monkeypatch.setenv("MFX_RENUMBER", mode)
        eng = BattleBatch(M, E, stream=torch.cuda.current_stream())
        eng.rollout_init([left, right], max_steps=24, eps=0.3, seed=77, stagger=True)
        eng.rollout_substeps(16)
        assert eng.rollout_path() == "k_rollout_bigq"
        eng.rollout_step(T)
        eng.rollout_check()
        dumps.append(_dump_rollout(eng, E, N))
        del eng
    for other in dumps[1:]:
        for (k, x), (_, y) in zip(dumps[0], other):
            assert torch.equal(x, y), k


def test_rollout_lds_step_matches_hbm_step(monkeypatch):
    """The few-env path's step staged in LDS (RolloutArgs::lds_step, the default) against the same step in
    HBM (MFX_LDS_STEP=0): 64 staggered 64x64 envs, 16 steps per launch, 432 steps (every env restarts):
    every output buffer and the per-call ids / positions / hp bit for bit."""
    import torch
    from mfrl_amd.battle import BattleBatch
    E, N, T = 64, 128, 432
    left, right = bd.block_positions(64, N)
    dumps = []
    for mode in ("0", "1"):
        monkeypatch.setenv("MFX_LDS_STEP", mode)
        eng = BattleBatch(64, E, stream=torch.cuda.current_stream())
        eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=1234, stagger=True)
        eng.rollout_substeps(16)
        assert eng.rollout_path() == "k_rollout_bigq"
        eng.rollout_step(T)
        eng.rollout_check()
        dumps.append(_dump_rollout(eng, E, N))
        del eng
    for (k, x), (_, y) in zip(dumps[0], dumps[1]):
        assert torch.equal(x, y), k


@pytest.mark.parametrize("E,S", [(8, 20), (8, 64), (64, 7), (64, 300), (100, 1)])
def test_rollout_few_pipe_matches_queue_step(E, S, monkeypatch):
    """The pipelined few-env form (RolloutArgs::few_pipe, the default for <= grid / 4 LDS-sized envs: a stepper
    workgroup per env keeps it in LDS and steps while the items observe its snapshot) against the queue kernel's
    step-after-items form (MFX_FEW_PIPE=0): staggered 64x64 envs, 432 steps (every env restarts), every output
    buffer and the per-call ids / positions / hp bit for bit -- E not a multiple of the 8 XCDs, 1 and 7 steps per
    launch included, and 300 (the pipelined form's launches run past the queue kernel's 64)."""
    import torch
    from mfrl_amd.battle import BattleBatch
    N, T = 128, 432
    left, right = bd.block_positions(64, N)
    dumps = []
    for mode in ("0", "1"):
        monkeypatch.setenv("MFX_FEW_PIPE", mode)
        eng = BattleBatch(64, E, stream=torch.cuda.current_stream())
        eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=4321, stagger=True)
        eng.rollout_substeps(S)
        assert eng.rollout_path() == "k_rollout_bigq"
        eng.rollout_step(T)
        eng.rollout_check()
        dumps.append(_dump_rollout(eng, E, N))
        del eng
    for (k, x), (_, y) in zip(dumps[0], dumps[1]):
        assert torch.equal(x, y), k


@pytest.mark.parametrize("E,S", [(8, 7), (20, 0), (20, 300)])
def test_rollout_few_pipe_one_workgroup_per_xcd(E, S, monkeypatch):
    """Forward progress without co-residency: the pipelined few-env form launched with ONE
    workgroup per XCD (MFX_BIGQ_GRID=8), as when other work on the device holds every other slot.  Each XCD's single
    workgroup claims its first env's stepper role, takes back every observation item of its own filings (few_steal)
    and observes them after its step (few_stolen), then -- once its launch steps are done -- claims the XCD's next env
    from the ticket wait (bigq_wait's kQClaim; E = 20: two or three envs per XCD) and skips the stolen slots.
    Against the queue kernel's step-after-items form (MFX_FEW_PIPE=0, full grid): every output buffer and the
    per-call ids / positions / hp bit for bit after 432 steps (every env restarts)."""
    import torch
    from mfrl_amd.battle import BattleBatch
    N, T = 128, 432
    left, right = bd.block_positions(64, N)
    dumps = []
    for mode, grid in (("0", None), ("1", "8")):
        monkeypatch.setenv("MFX_FEW_PIPE", mode)
        if grid:
            monkeypatch.setenv("MFX_BIGQ_GRID", grid)
        eng = BattleBatch(64, E, stream=torch.cuda.current_stream())
        eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=97, stagger=True)
        eng.rollout_substeps(S)
        assert eng.rollout_path() == "k_rollout_bigq"
        eng.rollout_step(T)
        eng.rollout_check()
        dumps.append(_dump_rollout(eng, E, N))
        del eng
        monkeypatch.delenv("MFX_BIGQ_GRID", raising=False)
    for (k, x), (_, y) in zip(dumps[0], dumps[1]):
        assert torch.equal(x, y), k


def test_rollout_bigq_queue_step_one_workgroup_per_xcd(monkeypatch):
    """The queue kernel's step-after-items form (MFX_FEW_PIPE=0) with one workgroup per XCD (MFX_BIGQ_GRID=8): its
    waits are only on work held by running workgroups of the same XCD, and a workgroup leaves once its XCD's env-steps
    of the launch are done (xcd_done), so one resident workgroup per XCD completes the launch.  Against the full
    grid, bit for bit, 12 staggered 64x64 envs, 20 steps per launch, 432 steps."""
    import torch
    from mfrl_amd.battle import BattleBatch
    N, T, E = 128, 432, 12
    left, right = bd.block_positions(64, N)
    monkeypatch.setenv("MFX_FEW_PIPE", "0")
    dumps = []
    for grid in (None, "8"):
        if grid:
            monkeypatch.setenv("MFX_BIGQ_GRID", grid)
        eng = BattleBatch(64, E, stream=torch.cuda.current_stream())
        eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=31, stagger=True)
        eng.rollout_substeps(20)
        assert eng.rollout_path() == "k_rollout_bigq"
        eng.rollout_step(T)
        eng.rollout_check()
        dumps.append(_dump_rollout(eng, E, N))
        del eng
    for (k, x), (_, y) in zip(dumps[0], dumps[1]):
        assert torch.equal(x, y), k


@pytest.mark.parametrize("map_size,agents,E,T,chunk", [(64, 128, 12, 432, "5"), (256, 4096, 16, 48, "6")])
def test_rollout_bigq_env_chunks_match_one_launch(monkeypatch, map_size, agents, E, T, chunk):
    """The queue kernel over env chunks (MFX_BIGQ_CHUNK: consecutive launches over envs [0, 4), [4, 8), ... with
    queues of their own -- the engine's form past ~640 MB of env state) against one launch over every env, bit for
    bit: every output buffer and the per-call state after T steps at 20 steps per launch (staggered envs)."""
    import torch
    from mfrl_amd.battle import BattleBatch
    left, right = bd.block_positions(map_size, agents // 2)
    monkeypatch.setenv("MFX_FEW_PIPE", "0")
    dumps = []
    for ch in ("0", chunk):
        monkeypatch.setenv("MFX_BIGQ_CHUNK", ch)
        eng = BattleBatch(map_size, E, stream=torch.cuda.current_stream())
        eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=37, stagger=True)
        eng.rollout_substeps(20)
        assert eng.rollout_path() == "k_rollout_bigq"
        eng.rollout_step(T)
        eng.rollout_check()
        dumps.append(_dump_rollout(eng, E, agents // 2))
        del eng
    for (k, x), (_, y) in zip(dumps[0], dumps[1]):
        assert torch.equal(x, y), k


def test_rollout_substeps_auto_choice():
    """rollout_substeps(0): the engine picks the steps per launch for its path and batch (BattleEngine::sub_steps):
    1024 for the pipelined few-env stepper (in practice the whole rollout_step), 2 for k_rollout below 96 envs per
    CU, 20 for the large-env queue kernel; an explicit value is reported as given (above 64 clamped to 64 off the
    pipelined path).  The results do not depend on it (test_rollout_substeps_match_single_steps
    and the few-env replays at 20 and 64 steps per launch)."""
    import torch
    from mfrl_amd.battle import BattleBatch
    cases = ((64, 256, 8, "k_rollout_bigq", 1024), (64, 256, 2048, "k_rollout", 2), (256, 4096, 16, "k_rollout_bigq", 20))
    for map_size, agents, E, path, want in cases:
        left, right = bd.block_positions(map_size, agents // 2)
        eng = BattleBatch(map_size, E, stream=torch.cuda.current_stream())
        eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=5)
        assert eng.rollout_path() == path, (E, eng.rollout_path())
        eng.rollout_substeps(0)
        assert eng.get_substeps() == want, (map_size, E, eng.get_substeps())
        eng.rollout_substeps(7)
        assert eng.get_substeps() == 7
        eng.rollout_substeps(300)
        assert eng.get_substeps() == (300 if want == 1024 else 64)
        eng.rollout_substeps(0)
        eng.rollout_step(3)
        eng.rollout_check()
        del eng


@pytest.mark.parametrize("E", [8, 64])
def test_rollout_two_engines_two_streams(E):
    """Two engines on two streams of one device, both on the pipelined few-env path, their launches enqueued back to
    back and running at once (the pipelined form is not serialised: it needs one resident workgroup per XCD, and a
    launch leaves an XCD once its work there is done) -- both finish without a stalled wait (rollout_check) and,
    seeded alike, leave identical buffers."""
    import torch
    from mfrl_amd.battle import BattleBatch
    N = 128
    left, right = bd.block_positions(64, N)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    engs = []
    for st in streams:
        eng = BattleBatch(64, E, stream=st)
        eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=2468, stagger=True)
        eng.rollout_substeps(0)
        assert eng.rollout_path() == "k_rollout_bigq"
        engs.append(eng)
    for _ in range(3):
        for eng in engs:
            eng.rollout_step(150)
    torch.cuda.synchronize()
    dumps = []
    for eng in engs:
        eng.rollout_check()
        dumps.append(_dump_rollout(eng, E, N))
    for (k, x), (_, y) in zip(dumps[0], dumps[1]):
        assert torch.equal(x, y), k
