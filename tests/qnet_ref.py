"""Test infrastructure: the Q network forward restated in numpy on the packed weight blob the HIP kernels
read (csrc/policy_kernels.hip), in float64 -- so a CPU test can pin the blob layout (im2col column order
(ky, kx, ci), NHWC flatten, K padding) against the torch module, and GPU tests can compare the kernels
against a float64 reference.  ValueNet._construct_net: examples/battle_model/algo/base.py:123-183."""
import numpy as np


def blocks(blob, offsets, F, A, use_mf):
    Fp, Ap = (F + 3) & ~3, (A + 3) & ~3
    Kc = 256 + 32 + (32 if use_mf else 0)
    shapes = [(64, 32), (32,), (288, 32), (32,), (2592, 256), (256,), (Fp, 32), (32,), (Ap, 64), (64,), (64, 32),
              (32,), (Kc, 128), (128,), (128, 64), (64,), (64, 32), (32,)]
    b = np.asarray(blob, dtype=np.float64)
    return [b[o:o + int(np.prod(s))].reshape(s) for o, s in zip(offsets, shapes)]


def forward(blob, offsets, F, A, use_mf, view, feat, prob=None):
    """view [n, 13, 13, 7], feat [n, F], prob [n, A] -> q [n, A] (float64)."""
    w1, b1, w2, b2, wd, bd, we, be, wp1, bp1, wp2, bp2, w2d, b2d, wo, bo, wq, bq = blocks(blob, offsets, F, A, use_mf)
    relu = lambda x: np.maximum(x, 0.0)
    v = np.asarray(view, dtype=np.float64)
    n = v.shape[0]
    # conv1: im2col columns in (ky, kx, ci) order; the 64th weight row is padding (zero)
    cols = np.stack([v[:, ky:ky + 11, kx:kx + 11, :] for ky in range(3) for kx in range(3)], axis=3)  # n,11,11,9,7
    c1 = relu(cols.reshape(n, 11, 11, 63) @ w1[:63] + b1)
    cols = np.stack([c1[:, ky:ky + 9, kx:kx + 9, :] for ky in range(3) for kx in range(3)], axis=3)    # n,9,9,9,32
    c2 = relu(cols.reshape(n, 9, 9, 288) @ w2 + b2)
    h_obs = relu(c2.reshape(n, 2592) @ wd + bd)
    f = np.zeros((n, we.shape[0]))
    f[:, :F] = feat
    h = [h_obs, relu(f @ we + be)]
    if use_mf:
        p = np.zeros((n, wp1.shape[0]))
        p[:, :A] = prob
        h.append(relu(relu(p @ wp1 + bp1) @ wp2 + bp2))
    x = relu(np.concatenate(h, axis=1) @ w2d + b2d)
    x = relu(x @ wo + bo)
    return (x @ wq + bq)[:, :A]
