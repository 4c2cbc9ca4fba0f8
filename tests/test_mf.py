"""Mean-field kernels: mean-action pooling, MF-Q target, MF-AC returns.

CPU part: the oracle's mean action equals what the reference loop recorded in the Battle fixtures;
the oracle's MF-Q target and MF-AC returns equal the outputs of the reference's own algo/ lines
(tests/golden/algo_*.npz, run under a tensorflow stub by tests/golden/make_algo_fixtures.py).
GPU part: the HIP kernels equal those fixtures and the oracle bit for bit (float64 / float32 as the
reference's numpy dtype rules dictate)."""
import os
import sys

import numpy as np
import pytest

import common

sys.path.insert(0, os.path.join(common.REPO, "oracle"))
import mf_oracle  # noqa: E402


def test_oracle_mean_action_matches_fixture():
    fx = np.load(os.path.join(common.GOLDEN, "battle40_s1.npz"))
    n = fx["e0_n"]
    acts = common.unpack_actions(fx, "e0_", n)
    for t in range(0, len(n), 37):
        for g in range(2):
            assert mf_oracle.mean_action(acts[t][g], 21)[0].tobytes() == fx["e0_mean_action"][t, g].tobytes()


def _fx(name):
    return np.load(os.path.join(common.GOLDEN, name))


def test_oracle_mfq_target_matches_reference():
    fx = _fx("algo_mfq_target.npz")
    for b in range(int(fx["n_batches"])):
        got = mf_oracle.mfq_target(fx["b%d_eq" % b], fx["b%d_tq" % b], fx["b%d_r" % b], fx["b%d_done" % b])
        assert got.tobytes() == fx["b%d_target" % b].tobytes(), b


def _episodes(fx):
    offs = np.concatenate([[0], np.cumsum(fx["lens"])]).astype(np.int64)
    return offs, [fx["rewards"][offs[e]:offs[e + 1]] for e in range(len(fx["lens"]))]


@pytest.mark.parametrize("numpy1", [True, False])
def test_oracle_mfac_returns_matches_reference(numpy1):
    """Both promotion rules against the reference's MFAC.train loop; they differ in most entries."""
    fx = _fx("algo_mfac_returns.npz")
    offs, eps = _episodes(fx)
    got = np.concatenate([mf_oracle.mfac_returns(r, v, numpy1=numpy1) for r, v in zip(eps, fx["value"])])
    want = fx["returns_numpy1" if numpy1 else "returns_nep50"]
    assert got.tobytes() == want.tobytes()
    assert (fx["returns_numpy1"] != fx["returns_nep50"]).sum() > len(want) // 2


def test_oracle_target_dtype_is_float64():
    rs = np.random.RandomState(0)
    out = mf_oracle.mfq_target(rs.randn(8, 21).astype(np.float32), rs.randn(8, 21).astype(np.float32),
                               rs.randn(8).astype(np.float32), rs.rand(8) < 0.3)
    assert out.dtype == np.float64


@pytest.mark.gpu
def test_mean_action_kernel():
    import torch
    from mfrl_amd.mf import mean_action
    rs = np.random.RandomState(1)
    B, cap = 37, 300
    counts = rs.randint(0, cap, size=B).astype(np.int32)
    counts[3] = 0
    acts = rs.randint(0, 21, size=(B, cap)).astype(np.int32)
    out = mean_action(torch.tensor(acts, device="cuda"), torch.tensor(counts, device="cuda"), 21).cpu().numpy()
    for b in range(B):
        if counts[b] == 0:
            assert np.isnan(out[b]).all()
        else:
            assert out[b].tobytes() == mf_oracle.mean_action(acts[b, :counts[b]], 21)[0].tobytes()


@pytest.mark.gpu
def test_mfq_target_kernel():
    import torch
    from mfrl_amd.mf import mfq_target
    rs = np.random.RandomState(2)
    M, A = 4096, 21
    eq = rs.randn(M, A).astype(np.float32)
    eq[5, :] = 1.0                     # ties -> first index
    eq[6, 3] = np.nan                  # NaN -> its index
    tq = rs.randn(M, A).astype(np.float32)
    r = rs.randn(M).astype(np.float32)
    d = rs.rand(M) < 0.2
    got = mfq_target(*(torch.tensor(x, device="cuda") for x in (eq, tq, r, d.astype(np.uint8)))).cpu().numpy()
    ref = mf_oracle.mfq_target(eq, tq, r, d)
    assert got.tobytes() == ref.tobytes()


@pytest.mark.gpu
def test_mfq_target_kernel_matches_reference_vectors():
    import torch
    from mfrl_amd.mf import mfq_target
    fx = _fx("algo_mfq_target.npz")
    for b in range(int(fx["n_batches"])):
        args = [torch.tensor(fx["b%d_%s" % (b, k)], device="cuda") for k in ("eq", "tq", "r")]
        d = torch.tensor(fx["b%d_done" % b].astype(np.uint8), device="cuda")
        got = mfq_target(*args, d).cpu().numpy()
        assert got.tobytes() == fx["b%d_target" % b].tobytes(), b


@pytest.mark.gpu
@pytest.mark.parametrize("numpy1", [True, False])
def test_mfac_returns_kernel_matches_reference_vectors(numpy1):
    import torch
    from mfrl_amd.mf import mfac_returns
    fx = _fx("algo_mfac_returns.npz")
    offs, _ = _episodes(fx)
    t = torch.tensor(fx["rewards"], device="cuda")
    mfac_returns(t, torch.tensor(offs, device="cuda"), torch.tensor(fx["value"], device="cuda"), 0.95, numpy1=numpy1)
    want = fx["returns_numpy1" if numpy1 else "returns_nep50"]
    assert t.cpu().numpy().tobytes() == want.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("numpy1", [True, False])
def test_mfac_returns_kernel(numpy1):
    import torch
    from mfrl_amd.mf import mfac_returns
    rs = np.random.RandomState(3)
    lens = rs.randint(1, 400, size=50)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    rew = rs.randn(offs[-1]).astype(np.float32)
    val = rs.randn(50).astype(np.float32)
    t = torch.tensor(rew, device="cuda")
    mfac_returns(t, torch.tensor(offs, device="cuda"), torch.tensor(val, device="cuda"), numpy1=numpy1)
    got = t.cpu().numpy()
    ref = np.concatenate([mf_oracle.mfac_returns(rew[offs[e]:offs[e + 1]], val[e], numpy1=numpy1) for e in range(50)])
    assert got.tobytes() == ref.tobytes()
