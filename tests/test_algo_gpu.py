"""mfrl_amd.algo on the GPU: the MF-Q target through the HIP kernel
against a torch float64 restatement of algo/base.py:192-220, act / train / soft update on device,
one self-play round on the single-env drop-in and on the batched engine (observations never leave
HBM); the HBM replay rings against the reference's own MemoryGroup outputs.  The networks' numerics
are PARITY UNPINNED (TensorFlow absent)."""
import numpy as np
import pytest
import torch

import magent
from mfrl_amd.algo import play as P
from mfrl_amd.algo import spawn_ai, tools

pytestmark = pytest.mark.gpu


def _env(map_size=20):
    env = magent.GridWorld("battle", map_size=map_size)
    return env, env.get_handles()


def test_calc_target_q_matches_restatement():
    torch.manual_seed(0)
    env, h = _env()
    m = spawn_ai("mfq", None, env, h[0], "mfq-me", 50)
    n = 37
    obs = torch.rand(n, 13, 13, 7, device="cuda")
    feat = torch.rand(n, 34, device="cuda")
    prob = torch.rand(n, 21, device="cuda")
    rew = torch.randn(n, device="cuda")
    done = torch.rand(n, device="cuda") < 0.3
    got = m.calc_target_q(obs=obs, feature=feat, prob=prob, rewards=rew, dones=done)
    with torch.no_grad():
        e_q = m.eval_net(obs, feat, prob)
        t_q = m.target_net(obs, feat, prob)
    q = t_q[torch.arange(n), torch.argmax(e_q, 1)].double()
    want = rew.double() + (1.0 - done.double()) * q * 0.95
    np.testing.assert_array_equal(got, want.cpu().numpy())


def test_soft_update_and_self_play_update():
    env, h = _env()
    a = spawn_ai("mfq", None, env, h[0], "a", 50)
    b = spawn_ai("mfq", None, env, h[1], "b", 50)
    with torch.no_grad():
        for p in a.eval_net.parameters():
            p.add_(1.0)
    t0 = [p.clone() for p in a.target_net.parameters()]
    a.update()
    for t, e, t_old in zip(a.target_net.parameters(), a.eval_net.parameters(), t0):
        assert torch.allclose(t, a.tau * e + (1 - a.tau) * t_old)
    r = tools.Runner.__new__(tools.Runner)
    r.models, r.tau = [a, b], 0.01
    b_old = [p.clone() for p in b.vars]
    r.self_play_update()
    for bv, av, bo in zip(b.vars, a.vars, b_old):
        assert torch.allclose(bv, 0.99 * av + 0.01 * bo)


@pytest.mark.parametrize("algo", ["mfq", "mfac"])
def test_single_env_round_trains(algo, tmp_path):
    np.random.seed(0)
    env, h = _env()
    models = [spawn_ai(algo, None, env, h[0], algo + "-me", 30), spawn_ai(algo, None, env, h[1], algo + "-op", 30)]
    max_nums, nums, mean_r, total_r = P.play(env, 0, 20, 30, h, models, print_every=10, eps=0.5, train=True)
    assert sum(max_nums) > 0 and all(np.isfinite(mean_r))
    models[0].save(str(tmp_path), 0)
    models[1].load(str(tmp_path), 0)


@pytest.mark.parametrize("algo", ["mfq", "mfac", "il", "ac"])
def test_batched_round_in_hbm(algo):
    from mfrl_amd.battle import BattleBatch
    np.random.seed(1)
    env, h = _env(24)
    models = [spawn_ai(algo, None, env, h[0], algo + "-me", 25), spawn_ai(algo, None, env, h[1], algo + "-op", 25)]
    eng = BattleBatch(24, 6, stream=torch.cuda.current_stream())
    max_nums, nums, mean_r, total_r = P.play_batched(eng, 0, 24, 25, models, print_every=10, eps=0.5, train=True,
                                                     left_id=0)
    assert max_nums[0] == 6 * 16 and max_nums[1] == 6 * 16       # 0.04 * 24^2 -> 4x4 block per side, 6 envs
    assert all(np.isfinite(mean_r)) and all(np.isfinite(total_r))


@pytest.mark.parametrize("algo", ["mfq", "il"])
def test_graph_train_matches_eager(algo):
    """train() as one HIP graph per minibatch (ValueNet.train_batches) against the reference-shaped
    eager loop (sample -> calc_target_q -> train -> update per minibatch): same np.random draws,
    same parameters afterwards (float tolerance: MIOpen may pick other conv algorithms)."""
    from mfrl_amd.algo.base import ValueNet as VN
    np.random.seed(3)
    torch.manual_seed(3)
    env, h = _env()
    m = spawn_ai(algo, None, env, h[0], algo + "-g", 30)
    opp = spawn_ai(algo, None, env, h[1], algo + "-o", 30)
    m.train = lambda: None                           # fill the replay only
    P.play(env, 0, 20, 30, h, [m, opp], print_every=100, eps=0.5, train=True)
    del m.train
    buf = m.replay_buffer
    buf.tight()
    batch_num = buf.get_batch_num()
    assert batch_num >= 6
    twin = spawn_ai(algo, None, env, h[0], algo + "-t", 30)      # same weights, fresh Adam state
    twin.eval_net.load_state_dict(m.eval_net.state_dict())
    twin.target_net.load_state_dict(m.target_net.state_dict())
    state = np.random.get_state()
    m.train_batches(buf, batch_num, use_mean=(algo == "mfq"))
    np.random.set_state(state)
    twin.graph_train = False
    twin.replay_buffer = buf
    for i in range(batch_num):                       # the eager loop of q_learning.py, same buffer
        s = buf.sample()
        if algo == "mfq":
            obs, feat, acts, prob, obs_n, feat_n, prob_n, rew, done, mask = s
            tq = twin.calc_target_q_dev(obs=obs_n, feature=feat_n, rewards=rew, dones=done, prob=prob_n)
            VN.train(twin, state=[obs, feat], target_q=tq, prob=prob, acts=acts, masks=mask)
        else:
            obs, feat, obs_n, feat_n, done, rew, acts, mask = s
            tq = twin.calc_target_q_dev(obs=obs_n, feature=feat_n, rewards=rew, dones=done)
            VN.train(twin, state=[obs, feat], target_q=tq, acts=acts, masks=mask)
        twin.update()
    for a, b in zip(m.vars, twin.vars):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)


def test_device_replay_matches_reference_fixture():
    """The HBM replay rings (device='cuda') against the reference's own MemoryGroup / EpisodesBuffer
    outputs (tests/golden/algo_replay.npz), bit for bit."""
    import test_algo_cpu
    test_algo_cpu._reference_replay_check("cuda")
