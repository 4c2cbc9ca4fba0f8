"""The hand-written HIP forward of the Q network (csrc/policy_kernels.hip, mfrl_amd.policy.QNetHIP) on the GPU.

* Against the torch module it was packed from (mfrl_amd.algo.nets.QNet = ValueNet._construct_net,
  algo/base.py:123-183) and against the float64 numpy restatement on the packed blob (tests/qnet_ref.py), on
  bench-shape batches: observations of a 64x64 rollout (~10^5 live agents).  Tolerance 1e-5 on the Q values
  (the north star's bound for float outputs); the greedy actions equal wherever the top two Q values are
  more than that apart.  Parity with the reference's TF1 network itself is unpinned: TensorFlow is absent.
* In the loop: a learned policy (one QNet per group, mean field) drives a rollout through
  mfx_qnet_act_rollout + mfx_battle_rollout_policy_step; every env is replayed on the C oracle with the
  actions the device chose, step by step (observations, rewards, mean actions, episode restarts).
"""
import numpy as np
import pytest

import battle_driver as bd
import common
import qnet_ref

pytestmark = pytest.mark.gpu


def _net(use_mf, seed):
    import torch
    from mfrl_amd.algo.nets import QNet
    torch.manual_seed(seed)
    net = QNet((13, 13, 7), (34,), 21, use_mf).cuda()
    with torch.no_grad():
        for p in net.parameters():
            p.add_(0.05 * torch.randn_like(p))
    return net


def _rollout_obs(E=4096, steps=60):
    """Live-agent rows (views, features, per-row group-0 mean action) of a 64x64 rollout after `steps` steps."""
    import torch
    from mfrl_amd.battle import BattleBatch
    left, right = bd.block_positions(64, 128)
    eng = BattleBatch(64, E, stream=torch.cuda.current_stream())
    eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=5, stagger=True)
    eng.rollout_step(steps)
    rc = eng.rowcap
    view = torch.empty((E, rc, 1183), dtype=torch.float32, device="cuda")
    feat = torch.empty((E, rc, 34), dtype=torch.float32, device="cuda")
    num = torch.empty((E, 2), dtype=torch.int32, device="cuda")
    mean = torch.empty((E, 2, 21), dtype=torch.float64, device="cuda")
    eng.rollout_copy("view", view, group=0)
    eng.rollout_copy("feature", feat, group=0)
    eng.rollout_copy("group_num", num)
    eng.rollout_copy("mean_action", mean)
    eng.sync()
    live = torch.arange(rc, device="cuda")[None, :] < num[:, 0:1]
    prob = mean[:, 0:1, :].expand(E, rc, 21).float()
    return view[live].reshape(-1, 13, 13, 7), feat[live], prob[live]


@pytest.mark.parametrize("use_mf", [False, True])
def test_qnet_forward_matches_torch_module(use_mf):
    import torch
    from mfrl_amd.policy import QNetHIP
    net = _net(use_mf, 11 + use_mf)
    view, feat, prob = _rollout_obs()
    n = view.shape[0]
    assert n > 50000
    hip = QNetHIP((13, 13, 7), (34,), 21, use_mf).load(net)
    q, act = hip.forward(view, feat, prob if use_mf else None)
    with torch.no_grad():
        want = net(view, feat, prob if use_mf else None)
    torch.cuda.synchronize()
    scale = max(1.0, float(want.abs().max()))
    err = float((q - want).abs().max())
    assert err <= 1e-5 * scale, (err, scale)
    top2 = torch.topk(want, 2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-5 * scale
    assert bool(clear.float().mean() > 0.99)
    assert torch.equal(act[clear].long(), torch.argmax(want, dim=1)[clear])
    # a sample of rows against the float64 restatement on the packed blob
    idx = torch.randperm(n, device="cuda")[:512]
    ref = qnet_ref.forward(hip.pack(net).cpu().double().numpy(), hip.offsets, 34, 21, use_mf,
                           view[idx].cpu().numpy(), feat[idx].cpu().numpy(), prob[idx].cpu().numpy() if use_mf else None)
    err64 = np.abs(q[idx].cpu().double().numpy() - ref).max()
    assert err64 <= 1e-5 * scale, err64


def test_qnet_forward_small_and_ragged_batches():
    """n = 1, 15, 17, 63, 65 (partial waves and workgroups) give the rows a full batch gives them."""
    import torch
    from mfrl_amd.policy import QNetHIP
    net = _net(True, 5)
    view, feat, prob = _rollout_obs(E=256, steps=30)
    hip = QNetHIP((13, 13, 7), (34,), 21, True).load(net)
    q_all, a_all = hip.forward(view[:200], feat[:200], prob[:200])
    for n in (1, 15, 17, 63, 65):
        q, a = hip.forward(view[:n], feat[:n], prob[:n])
        torch.cuda.synchronize()
        assert torch.equal(q, q_all[:n]) and torch.equal(a, a_all[:n]), n


def test_learned_policy_rollout_matches_oracle(monkeypatch):
    """Two mean-field QNets (one per group) in the loop on the fused k_rollout: per step the HIP forward
    acts on the observation in the rollout buffers, k_rollout (kMode 1) steps with those actions and
    observes.  Every env replayed on the C oracle with the device's actions: views, features, rewards and
    mean actions bit for bit, restarts included; the device's actions are the torch module's argmax on
    the device's own observation wherever its top two Q values are apart."""
    import torch
    from mfrl_amd.battle import BattleBatch
    from mfrl_amd.policy import QNetHIP
    monkeypatch.setenv("MFX_SMALL_E", "0")               # 3 envs on the fused path
    E, T, max_steps, VF, F = 3, 70, 30, 1183, 34
    left, right = bd.block_positions(64, 128)
    eng = BattleBatch(64, E, stream=torch.cuda.current_stream())
    eng.rollout_init([left, right], max_steps=max_steps, eps=0.0, seed=1, stagger=False)
    assert eng.rollout_path() == "k_rollout"
    nets = [_net(True, 21), _net(True, 22)]
    pols = [QNetHIP((13, 13, 7), (34,), 21, True).load(n) for n in nets]
    rc = eng.rowcap
    oracles = []
    for e in range(E):
        env, h = common.battle_env(common.ORACLE_LIB, 64)
        env.reset()
        env.add_agents(h[0], method="custom", pos=left)
        env.add_agents(h[1], method="custom", pos=right)
        oracles.append([env, h, 0])
    eng.rollout_policy_observe()

    def grab():
        out = {}
        for g in range(2):
            out["view%d" % g] = torch.empty((E, rc, VF), dtype=torch.float32, device="cuda")
            out["feat%d" % g] = torch.empty((E, rc, F), dtype=torch.float32, device="cuda")
            eng.rollout_copy("view", out["view%d" % g], group=g)
            eng.rollout_copy("feature", out["feat%d" % g], group=g)
        out["mean"] = torch.empty((E, 2, 21), dtype=torch.float64, device="cuda")
        eng.rollout_copy("mean_action", out["mean"])
        eng.sync()
        return out

    obs = grab()
    restarts, checked = 0, 0
    for t in range(T):
        for g in range(2):
            pols[g].act_rollout(eng, g)
        act = torch.empty((E, 2, rc), dtype=torch.int32, device="cuda")
        eng.rollout_copy("actions", act)
        eng.sync()
        actn = act.cpu().numpy()
        # the device's actions are the module's greedy actions on the device's observation
        for g in range(2):
            for e in range(E):
                n = len(oracles[e][0].get_agent_id(oracles[e][1][g]))
                if not n:
                    continue
                prob = obs["mean"][e, g].float().expand(n, 21)
                with torch.no_grad():
                    qv = nets[g](obs["view%d" % g][e, :n].reshape(n, 13, 13, 7), obs["feat%d" % g][e, :n], prob)
                top2 = torch.topk(qv, min(2, qv.shape[1]), dim=1).values
                clear = ((top2[:, 0] - top2[:, 1]) > 1e-5).cpu().numpy()
                want = torch.argmax(qv, 1).cpu().numpy()
                assert np.array_equal(actn[e, g, :n][clear], want[clear]), (t, e, g)
                checked += int(clear.sum())
        eng.rollout_policy_step()
        nxt = grab()
        rew = torch.empty((E, 2, rc), dtype=torch.float32, device="cuda")
        eng.rollout_copy("rewards", rew)
        eng.sync()
        for e, st in enumerate(oracles):
            env, h, _ = st
            acts = []
            for g in range(2):
                n = len(env.get_agent_id(h[g]))
                acts.append(np.ascontiguousarray(actn[e, g, :n]))
            for g in range(2):
                env.set_action(h[g], acts[g])
            done = env.step()
            for g in range(2):
                rw = env.get_reward(h[g])
                assert rew[e, g, :len(rw)].cpu().numpy().tobytes() == rw.tobytes(), (t, e, g, "reward")
            env.clear_dead()
            st[2] += 1
            restart = done or st[2] >= max_steps
            for g in range(2):
                n = len(acts[g])
                want = np.bincount(acts[g], minlength=21) / n if n else np.full(21, np.nan)
                got = nxt["mean"][e, g].cpu().numpy()
                if restart:
                    assert not got.any(), (t, e, g, "mean reset")          # former_act_prob = 0 again
                else:
                    assert np.array_equal(got, want, equal_nan=True), (t, e, g, "mean")
            if restart:
                st[2] = 0
                restarts += 1
                env.reset()
                env.add_agents(h[0], method="custom", pos=left)
                env.add_agents(h[1], method="custom", pos=right)
            for g in range(2):
                v, f = env.get_observation(h[g])
                n = len(v)
                assert nxt["view%d" % g][e, :n].cpu().numpy().tobytes() == v.reshape(n, VF).tobytes(), (t, e, g)
                assert nxt["feat%d" % g][e, :n].cpu().numpy().tobytes() == f.tobytes(), (t, e, g)
        obs = nxt
    eng.rollout_check()
    assert restarts >= E and checked > 1000


# ---------------------------------------------------------------------------------------------------------------
# the actor-critic forward (ActorCritic / MFAC, algo/ac.py:48-98, :219-276) on k_acnet
# ---------------------------------------------------------------------------------------------------------------
def _acnet(use_mf, seed):
    import torch
    from mfrl_amd.algo.nets import ACNet
    torch.manual_seed(seed)
    net = ACNet((13, 13, 7), (34,), 21, use_mf=use_mf).cuda()
    with torch.no_grad():
        for p in net.parameters():
            p.add_(0.02 * torch.randn_like(p))
    return net


@pytest.mark.parametrize("use_mf", [False, True])
def test_acnet_forward_matches_torch_module(use_mf):
    """k_acnet on bench-shape rows (~10^5 live agents of a 64x64 rollout) against the torch ACNet it was packed
    from: the clipped softmax policy and the value within 1e-5 (scaled by the value's magnitude); a sample of
    rows against the float64 restatement on the packed blob; every sampled action equals the host restatement of
    the draw on the kernel's own policy rows.  Parity with TF's network itself is unpinned (TensorFlow absent)."""
    import acnet_ref
    import torch
    from mfrl_amd.policy import ACNetHIP
    net = _acnet(use_mf, 31 + use_mf)
    view, feat, prob = _rollout_obs()
    n = view.shape[0]
    assert n > 50000
    hip = ACNetHIP((13, 13, 7), (34,), 21, use_mf).load(net)
    pol, val, act = hip.forward(view, feat, prob, want_value=True, seed=77, step=5)
    with torch.no_grad():
        wp, wv = net(view, feat, prob if use_mf else None)
    torch.cuda.synchronize()
    perr = float((pol - wp).abs().max())
    scale = max(1.0, float(wv.abs().max()))
    verr = float((val - wv).abs().max())
    assert perr <= 1e-5, perr
    assert verr <= 1e-5 * scale, (verr, scale)
    assert float(wp.max(1).values.mean()) < 0.999            # (a policy that is not one-hot everywhere)
    want = acnet_ref.draw(pol.cpu().numpy(), 77, 5, 0, np.arange(n))
    assert np.array_equal(act.cpu().numpy(), want)
    idx = torch.randperm(n, device="cuda")[:512]
    rp, rv = acnet_ref.forward(hip.pack(net).cpu().double().numpy(), hip.offsets, 1183, 34, 21, use_mf,
                               view[idx].cpu().numpy(), feat[idx].cpu().numpy(), prob[idx].cpu().numpy())
    assert np.abs(pol[idx].cpu().double().numpy() - rp).max() <= 1e-5
    assert np.abs(val[idx].cpu().double().numpy() - rv).max() <= 1e-5 * scale
    # the draw follows the policy: mean sampled-action probability against the expected one
    p_of = pol.gather(1, act.long()[:, None]).squeeze(1)
    assert abs(float(p_of.mean()) - float((pol * pol).sum(1).mean())) < 0.01


@pytest.mark.parametrize("use_mf", [False, True])
def test_acnet_input_support_is_bit_identical(use_mf):
    """The view layer over the engine's view support only (mfx_acnet_set_input_support with
    mfx_battle_view_support: 903 of the 1,183 inputs, the rest never written by the observation) gives the dense
    forward's policy, value and draw bit for bit, on bench-shape rollout rows -- whose unsupported inputs are
    checked to be exactly zero -- and on random rows zeroed outside a random support (other gaps in the packed
    order, ragged n)."""
    import torch
    from mfrl_amd.battle import BattleBatch
    from mfrl_amd.policy import ACNetHIP
    net = _acnet(use_mf, 51 + use_mf)
    view, feat, prob = _rollout_obs(E=2048, steps=45)
    n = view.shape[0]
    mask = BattleBatch(64, 4, stream=torch.cuda.current_stream()).view_support(0)
    assert int(mask.sum()) == 903
    off = torch.from_numpy(mask == 0).cuda()
    assert not view.reshape(n, -1)[:, off].any()              # the observation never writes them
    hip = ACNetHIP((13, 13, 7), (34,), 21, use_mf).load(net)
    dense = hip.forward(view, feat, prob, want_value=True, seed=9, step=2)
    hip.set_input_support(mask)
    assert hip.input_support_size() == 903
    packed = hip.forward(view, feat, prob, want_value=True, seed=9, step=2)
    torch.cuda.synchronize()
    for a, b in zip(dense, packed):
        assert torch.equal(a, b)
    # an arbitrary support; support cleared again -> dense
    rng = np.random.RandomState(3)
    rmask = (rng.rand(1183) < 0.55).astype(np.uint8)
    m = 517
    v = torch.randn(m, 1183, device="cuda") * torch.from_numpy(rmask).cuda().float()
    hip.set_input_support(rmask)
    assert hip.input_support_size() == int(rmask.sum())
    packed = hip.forward(v, feat[:m], prob[:m], want_value=True, seed=1, step=7)
    hip.load(_acnet(use_mf, 61))                              # new weights: the packed image is remade
    packed2 = hip.forward(v, feat[:m], prob[:m], want_value=True, seed=1, step=7)
    hip.set_input_support(None)
    assert hip.input_support_size() == 0
    dense2 = hip.forward(v, feat[:m], prob[:m], want_value=True, seed=1, step=7)
    hip.load(net)
    dense = hip.forward(v, feat[:m], prob[:m], want_value=True, seed=1, step=7)
    torch.cuda.synchronize()
    for a, b, c, d in zip(dense, packed, dense2, packed2):
        assert torch.equal(a, b) and torch.equal(c, d)
    assert not torch.equal(dense[0], dense2[0])


def test_acnet_forward_small_and_ragged_batches():
    """n = 1, 15, 17, 63, 65 give the rows (policy, value, draw) a full batch gives them."""
    import torch
    from mfrl_amd.policy import ACNetHIP
    net = _acnet(True, 9)
    view, feat, prob = _rollout_obs(E=256, steps=30)
    hip = ACNetHIP((13, 13, 7), (34,), 21, True).load(net)
    p_all, v_all, a_all = hip.forward(view[:200], feat[:200], prob[:200], want_value=True, seed=3, step=1)
    for n in (1, 15, 17, 63, 65):
        p, v, a = hip.forward(view[:n], feat[:n], prob[:n], want_value=True, seed=3, step=1)
        torch.cuda.synchronize()
        assert torch.equal(p, p_all[:n]) and torch.equal(v, v_all[:n]) and torch.equal(a, a_all[:n]), n


def test_mfac_policy_rollout_matches_oracle(monkeypatch):
    """Two MFAC networks (one per group) in the loop on the fused k_rollout: per step mfx_acnet_act_rollout
    samples every live agent's action on the device from the observation in the rollout buffers (nothing read
    back), k_rollout (kMode 1) steps with them and observes.  The device's actions equal the host restatement
    of the draw on the kernel's policy rows for the same observation (row e * rowcap + j, group g, the step);
    every env is replayed on the C oracle with those actions: views, features, rewards, mean actions bit for
    bit, restarts included."""
    import acnet_ref
    import torch
    from mfrl_amd.battle import BattleBatch
    from mfrl_amd.policy import ACNetHIP
    monkeypatch.setenv("MFX_SMALL_E", "0")
    E, T, max_steps, VF, F, seed = 3, 70, 30, 1183, 34, 4242
    left, right = bd.block_positions(64, 128)
    eng = BattleBatch(64, E, stream=torch.cuda.current_stream())
    eng.rollout_init([left, right], max_steps=max_steps, eps=0.0, seed=1, stagger=False)
    assert eng.rollout_path() == "k_rollout"
    pols = [ACNetHIP((13, 13, 7), (34,), 21, True).load(_acnet(True, 40 + g)) for g in range(2)]
    rc = eng.rowcap
    oracles = []
    for e in range(E):
        env, h = common.battle_env(common.ORACLE_LIB, 64)
        env.reset()
        env.add_agents(h[0], method="custom", pos=left)
        env.add_agents(h[1], method="custom", pos=right)
        oracles.append([env, h, 0])
    eng.rollout_policy_observe()

    def grab():
        out = {}
        for g in range(2):
            out["view%d" % g] = torch.empty((E, rc, VF), dtype=torch.float32, device="cuda")
            out["feat%d" % g] = torch.empty((E, rc, F), dtype=torch.float32, device="cuda")
            eng.rollout_copy("view", out["view%d" % g], group=g)
            eng.rollout_copy("feature", out["feat%d" % g], group=g)
        out["mean"] = torch.empty((E, 2, 21), dtype=torch.float64, device="cuda")
        eng.rollout_copy("mean_action", out["mean"])
        eng.sync()
        return out

    obs = grab()
    restarts = 0
    for t in range(T):
        for g in range(2):
            pols[g].act_rollout(eng, g, seed, t)
        act = torch.empty((E, 2, rc), dtype=torch.int32, device="cuda")
        eng.rollout_copy("actions", act)
        eng.sync()
        actn = act.cpu().numpy()
        for g in range(2):
            for e in range(E):
                n = len(oracles[e][0].get_agent_id(oracles[e][1][g]))
                if not n:
                    continue
                pol, _, _ = pols[g].forward(obs["view%d" % g][e, :n], obs["feat%d" % g][e, :n], want_act=False)
                want = acnet_ref.draw(pol.cpu().numpy(), seed, t, g, e * rc + np.arange(n))
                assert np.array_equal(actn[e, g, :n], want), (t, e, g)
        eng.rollout_policy_step()
        nxt = grab()
        rew = torch.empty((E, 2, rc), dtype=torch.float32, device="cuda")
        eng.rollout_copy("rewards", rew)
        eng.sync()
        for e, st in enumerate(oracles):
            env, h, _ = st
            acts = [np.ascontiguousarray(actn[e, g, :len(env.get_agent_id(h[g]))]) for g in range(2)]
            for g in range(2):
                env.set_action(h[g], acts[g])
            done = env.step()
            for g in range(2):
                rw = env.get_reward(h[g])
                assert rew[e, g, :len(rw)].cpu().numpy().tobytes() == rw.tobytes(), (t, e, g, "reward")
            env.clear_dead()
            st[2] += 1
            restart = done or st[2] >= max_steps
            for g in range(2):
                n = len(acts[g])
                want = np.bincount(acts[g], minlength=21) / n if n else np.full(21, np.nan)
                got = nxt["mean"][e, g].cpu().numpy()
                if restart:
                    assert not got.any(), (t, e, g, "mean reset")
                else:
                    assert np.array_equal(got, want, equal_nan=True), (t, e, g, "mean")
            if restart:
                st[2] = 0
                restarts += 1
                env.reset()
                env.add_agents(h[0], method="custom", pos=left)
                env.add_agents(h[1], method="custom", pos=right)
            for g in range(2):
                v, f = env.get_observation(h[g])
                n = len(v)
                assert nxt["view%d" % g][e, :n].cpu().numpy().tobytes() == v.reshape(n, VF).tobytes(), (t, e, g)
                assert nxt["feat%d" % g][e, :n].cpu().numpy().tobytes() == f.tobytes(), (t, e, g)
        obs = nxt
    eng.rollout_check()
    assert restarts >= E


@pytest.mark.parametrize("E", [1, 63, 64, 65, 8192, 131072])
def test_rollout_rows_match_numpy(E):
    """The compact row list of act_rollout (two-level scan over 64-env chunks) at up to the bench's
    131072 envs: every row index and the count against numpy, counts capped at rowcap, empty envs included."""
    import ctypes
    import torch
    from mfrl_amd import check, lib
    from mfrl_amd.policy import rows_scratch
    G, rowcap = 2, 128
    rng = np.random.RandomState(E)
    counts = rng.randint(0, rowcap + 40, size=(E, G)).astype(np.int32)
    counts[rng.rand(E) < 0.1, 1] = 0
    d_counts = torch.from_numpy(counts).cuda()
    buf = torch.full((rows_scratch(E, rowcap),), -7, dtype=torch.int32, device="cuda")
    L = lib()
    L.mfx_rollout_rows.restype = ctypes.c_int
    P = ctypes.c_void_p
    check(L.mfx_rollout_rows(P(d_counts.data_ptr()), E, G, 1, rowcap, P(buf.data_ptr()),
                             P(buf.data_ptr() + 4 * E * rowcap), P(torch.cuda.current_stream().cuda_stream)),
          "mfx_rollout_rows")
    got = buf.cpu().numpy()
    n = np.minimum(counts[:, 1], rowcap)
    want = np.concatenate([e * rowcap + np.arange(k) for e, k in enumerate(n)]) if n.sum() else np.zeros(0, np.int32)
    assert got[E * rowcap] == n.sum()
    assert np.array_equal(got[:len(want)], want)
