"""The packed weight blob of the HIP Q-network forward (mfrl_amd.policy.pack_qnet) on the CPU: the numpy
restatement of the kernels' arithmetic on that blob (tests/qnet_ref.py) reproduces the torch module
(mfrl_amd.algo.nets.QNet = ValueNet._construct_net, algo/base.py:123-183) -- so the layout the kernels read
(im2col order, NHWC flatten, padding) is the network's.  The kernels themselves: tests/test_policy_gpu.py."""
import numpy as np
import pytest
import torch

import qnet_ref


@pytest.mark.parametrize("use_mf", [False, True])
def test_packed_blob_is_the_torch_network(use_mf):
    from mfrl_amd.algo.nets import QNet
    from mfrl_amd.policy import blob_layout, pack_qnet
    torch.manual_seed(3)
    F, A, n = 34, 21, 37
    net = QNet((13, 13, 7), (F,), A, use_mf).double()
    for p in net.parameters():            # non-zero biases, so a misplaced bias block shows
        with torch.no_grad():
            p.add_(0.05 * torch.randn_like(p))
    rng = np.random.RandomState(0)
    view = (rng.rand(n, 13, 13, 7) < 0.3) * rng.rand(n, 13, 13, 7)
    feat = rng.rand(n, F)
    prob = rng.dirichlet(np.ones(A), n) if use_mf else None
    with torch.no_grad():
        want = net(torch.tensor(view), torch.tensor(feat), torch.tensor(prob) if use_mf else None).numpy()
    layout = blob_layout(F, A, use_mf)
    blob = pack_qnet(net, F, A, use_mf, layout).double().numpy()
    got = qnet_ref.forward(blob, layout[1], F, A, use_mf, view, feat, prob)
    # float32 weights in the blob: the network itself rounded to float32, so agreement to ~1e-6
    assert np.abs(got - want).max() < 1e-5 * max(1.0, np.abs(want).max()), np.abs(got - want).max()
    assert np.array_equal(np.argmax(got, 1)[np.sort(got, 1)[:, -1] - np.sort(got, 1)[:, -2] > 1e-5],
                          np.argmax(want, 1)[np.sort(got, 1)[:, -1] - np.sort(got, 1)[:, -2] > 1e-5])


@pytest.mark.parametrize("use_mf", [False, True])
def test_packed_acnet_blob_is_the_torch_network(use_mf):
    """The actor-critic blob (mfrl_amd.policy.pack_acnet) restated in float64 (tests/acnet_ref.py) reproduces
    the torch ACNet (ActorCritic / MFAC._create_network, algo/ac.py:48-98, :219-276): policy and value."""
    import acnet_ref
    from mfrl_amd.algo.nets import ACNet
    from mfrl_amd.policy import acnet_layout, pack_acnet
    torch.manual_seed(4)
    F, A, n, V = 34, 21, 41, 13 * 13 * 7
    net = ACNet((13, 13, 7), (F,), A, use_mf=use_mf).double()
    for p in net.parameters():
        with torch.no_grad():
            p.add_(0.02 * torch.randn_like(p))
    rng = np.random.RandomState(1)
    view = (rng.rand(n, 13, 13, 7) < 0.3) * rng.rand(n, 13, 13, 7)
    feat = rng.rand(n, F)
    prob = rng.dirichlet(np.ones(A), n)
    with torch.no_grad():
        pol, val = net(torch.tensor(view), torch.tensor(feat), torch.tensor(prob) if use_mf else None)
    layout = acnet_layout(V, F, A, use_mf)
    blob = pack_acnet(net, V, F, A, use_mf, layout).double().numpy()
    gp, gv = acnet_ref.forward(blob, layout[1], V, F, A, use_mf, view, feat, prob)
    assert np.abs(gp - pol.numpy()).max() < 1e-5
    assert np.abs(gv - val.numpy()).max() < 1e-5 * max(1.0, np.abs(val.numpy()).max())


def test_acnet_draw_restatement():
    """The draw's host restatement: a one-hot policy always yields its action, u spreads over [0, 1), and the
    frequencies of a fixed policy follow it (the reference's tf.multinomial(log p) samples a with p[a] / sum p)."""
    import acnet_ref
    A, n = 21, 200000
    u = acnet_ref.uniforms(7, 3, 1, np.arange(n))
    assert u.dtype == np.float32 and 0.0 <= u.min() and u.max() < 1.0 and abs(float(u.mean()) - 0.5) < 0.01
    one = np.full((5, A), 1e-10, dtype=np.float32)
    one[np.arange(5), [0, 3, 7, 20, 11]] = 1.0
    assert acnet_ref.draw(one, 1, 2, 0, np.arange(5)).tolist() == [0, 3, 7, 20, 11]
    p = np.random.RandomState(0).dirichlet(np.ones(A)).astype(np.float32)
    got = np.bincount(acnet_ref.draw(np.tile(p, (n, 1)), 9, 0, 0, np.arange(n)), minlength=A) / n
    assert np.abs(got - p / p.sum()).max() < 0.005
