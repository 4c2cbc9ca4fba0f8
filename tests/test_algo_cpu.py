"""mfrl_amd.algo on the CPU: the device replay buffers (run with device='cpu') against the outputs of
the reference's own MemoryGroup / EpisodesBuffer (tests/golden/algo_replay.npz, recorded by
make_algo_fixtures.py under a tensorflow stub) and against the numpy restatement
oracle/algo_oracle.py, under the same np.random stream; network shapes; the epsilon schedule.  The
networks themselves stay PARITY UNPINNED (their numerics need TensorFlow)."""
import os
import sys

import numpy as np
import pytest
import torch

import common

sys.path.insert(0, os.path.join(common.REPO, "oracle"))
import algo_oracle  # noqa: E402
from mfrl_amd.algo import nets, tools  # noqa: E402

V, F, A = (13, 13, 7), (34,), 21


def _episode(rng, n_agents, steps, die_p):
    """Per-step pushes of one group: ids shrink as agents die (clear_dead), like the real loop."""
    ids = np.arange(n_agents, dtype=np.int64) * 3 + 5
    pushes = []
    for _ in range(steps):
        if len(ids) == 0:
            break
        m = len(ids)
        alive = rng.random(m) > die_p
        pushes.append(dict(ids=ids.copy(), obs=rng.random((m,) + V, dtype=np.float32),
                           feat=rng.random((m,) + F, dtype=np.float32), acts=rng.integers(0, A, m).astype(np.int32),
                           rewards=rng.standard_normal(m).astype(np.float32), alives=alive,
                           prob=rng.random((m, A), dtype=np.float32)))
        ids = ids[alive]
    return pushes


@pytest.mark.parametrize("use_mean,sub_len,max_len", [(True, 400, 5000), (False, 400, 700), (True, 7, 5000),
                                                     (True, 400, 300)])
def test_memory_group_matches_oracle(use_mean, sub_len, max_len):
    rng = np.random.default_rng(3)
    dev = tools.MemoryGroup(V, F, A, max_len, 64, sub_len, use_mean=use_mean, device="cpu")
    ora = algo_oracle.MemoryGroupOracle(V, F, A, max_len, 64, sub_len, use_mean)
    for ep in range(3):                               # three episodes: the rings wrap at max_len 700
        pushes = _episode(rng, 40, 25, 0.04)
        for p in pushes:
            dev.push(state=[p["obs"], p["feat"]], acts=p["acts"], rewards=p["rewards"], alives=p["alives"],
                     ids=p["ids"], prob=p["prob"])
            ora.push(p["ids"], p["obs"], p["feat"], p["acts"], p["rewards"], p["alives"], p["prob"])
        np.random.seed(100 + ep)
        dev.tight()
        np.random.seed(100 + ep)
        ora.tight()
        assert dev.get_batch_num() == ora.get_batch_num()
        for b in range(4):
            np.random.seed(1000 * ep + b)
            got = dev.sample()
            np.random.seed(1000 * ep + b)
            want = ora.sample()
            if use_mean:
                names = ("obs", "feat", "act", "prob", "obs_next", "feat_next", "prob_next", "rew", "done", "mask")
            else:
                names = ("obs", "feat", "obs_next", "feat_next", "done", "rew", "act", "mask")
            assert len(got) == len(names)
            for name, g in zip(names, got):
                np.testing.assert_array_equal(g.numpy(), want[name], err_msg=name)


def test_episodes_buffer_groups_like_the_reference():
    rng = np.random.default_rng(5)
    pushes = _episode(rng, 12, 6, 0.1)
    buf = tools.EpisodesBuffer(use_mean=True, device="cpu")
    np.random.seed(9)
    for p in pushes:
        buf.push(state=[p["obs"], p["feat"]], acts=p["acts"], rewards=p["rewards"], alives=p["alives"],
                 ids=p["ids"], prob=p["prob"])
    rows, counts = buf.batch()
    np.random.seed(9)
    order = algo_oracle.episodes_order([p["ids"] for p in pushes])
    want_rew = np.concatenate([[pushes[p]["rewards"][j] for p, j in rs] for _, rs in order])
    want_obs = np.stack([pushes[p]["obs"][j] for _, rs in order for p, j in rs])
    assert counts.tolist() == [len(rs) for _, rs in order]
    np.testing.assert_array_equal(rows["rew"].numpy(), want_rew)
    np.testing.assert_array_equal(rows["obs"].numpy(), want_obs)


def test_network_shapes_and_flatten_order():
    torch.manual_seed(0)
    q = nets.QNet(V, F, A, use_mf=True)
    v = torch.rand(5, *V)
    out = q(v, torch.rand(5, *F), torch.rand(5, A))
    assert out.shape == (5, A)
    assert q.dense_obs.in_features == 9 * 9 * 32
    # the flatten is NHWC (TF order): channel fastest
    x = torch.nn.functional.relu(q.conv2(torch.nn.functional.relu(q.conv1(v.permute(0, 3, 1, 2)))))
    flat = x.permute(0, 2, 3, 1).reshape(5, -1)
    assert torch.equal(flat[:, :32], x[:, :, 0, 0])
    for mf_ in (False, True):
        ac = nets.ACNet(V, F, A, use_mf=mf_)
        pol, val = ac(v, torch.rand(5, *F), torch.rand(5, A))
        assert pol.shape == (5, A) and val.shape == (5,)
        assert torch.allclose(pol.sum(1), torch.ones(5), atol=1e-5)
        assert float(pol.detach().min()) >= 1e-10


def test_linear_decay_schedule():
    from mfrl_amd.train_battle import linear_decay
    x, y = [0, 1600, 2000], [1, 0.2, 0.1]
    assert linear_decay(0, x, y) == 1
    assert abs(linear_decay(800, x, y) - 0.6) < 1e-12
    assert abs(linear_decay(1600, x, y) - 0.2) < 1e-12
    assert abs(linear_decay(2000, x, y) - 0.1) < 1e-12


def _reference_replay_check(device):
    """The device replay buffers against the reference's own MemoryGroup / EpisodesBuffer outputs
    (tests/golden/algo_replay.npz, recorded by make_algo_fixtures.py from algo/tools.py:26-362):
    every sample() batch bit for bit under the same seeded np.random stream, get_batch_num, and the
    EpisodesBuffer per-agent order, rewards, views and probs."""
    sys.path.insert(0, common.GOLDEN)
    import make_algo_fixtures as mk
    fx = np.load(os.path.join(common.GOLDEN, "algo_replay.npz"))
    V, F, A = mk.REPLAY_V, mk.REPLAY_F, mk.REPLAY_A
    for ci, (use_mean, sub_len, max_len) in enumerate(mk.REPLAY_CASES):
        key = "c%d_" % ci
        mg = tools.MemoryGroup(V, F, A, max_len, 64, sub_len, use_mean=use_mean, device=device)
        pushes = mk.replay_pushes(ci)
        k = 0
        for ep in range(3):
            for e, p in pushes:
                if e == ep:
                    mg.push(state=[p["obs"], p["feat"]], acts=p["acts"], rewards=p["rewards"], alives=p["alives"],
                            ids=p["ids"], prob=p["prob"])
            np.random.seed(100 + ep)
            mg.tight()
            assert mg.get_batch_num() == fx[key + "nbatch"][ep], (ci, ep)
            for b in range(2):
                np.random.seed(1000 * ep + b)
                got = mg.sample()
                for j, g in enumerate(got):
                    want = fx[key + "s%d_%d" % (k, j)]
                    g = g.cpu().numpy()
                    assert g.dtype == want.dtype and g.shape == want.shape, (ci, k, j)
                    assert g.tobytes() == want.tobytes(), (ci, ep, b, j)
                k += 1
        assert k == int(fx[key + "nsample"])
    eb = tools.EpisodesBuffer(use_mean=True, device=device)
    np.random.seed(9)
    for p in mk.episodes_pushes():
        eb.push(state=[p["obs"], p["feat"]], acts=p["acts"], rewards=p["rewards"], alives=p["alives"], ids=p["ids"],
                prob=p["prob"])
    rows, counts = eb.batch()
    assert counts.cpu().numpy().tolist() == fx["eb_counts"].tolist()
    assert rows["rew"].cpu().numpy().tobytes() == fx["eb_rewards"].tobytes()
    assert rows["obs"].cpu().numpy().tobytes() == fx["eb_obs"].astype(np.float32).tobytes()
    assert rows["prob"].cpu().numpy().tobytes() == fx["eb_probs"].astype(np.float32).tobytes()


def test_replay_matches_reference_fixture():
    _reference_replay_check("cpu")
