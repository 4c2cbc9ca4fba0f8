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
