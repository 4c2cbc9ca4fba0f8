"""Test infrastructure: the actor-critic forward restated in numpy (float64) on the packed weight blob the HIP
kernel reads (csrc/acnet_kernels.hip, mfrl_amd.policy.pack_acnet), and the kernel's draw restated in float32.

ActorCritic._create_network: examples/battle_model/algo/ac.py:48-98; MFAC._create_network: :219-276; the act,
tf.multinomial(log(policy)): :43-46 / :213-217.  The draw is not the reference's RNG (TensorFlow is absent and its
stream is not reproducible here): it is the device's counter-hash uniform, restated exactly, applied to a given
float32 policy row."""
import numpy as np

_U32 = np.uint32


def blocks(blob, offsets, V, F, A, use_mf):
    Vp, Fp, Ap = (V + 3) & ~3, (F + 3) & ~3, (A + 3) & ~3
    mf, ac = (1, 0) if use_mf else (0, 1)
    shapes = [(Vp, 256), (256,), (Fp, 256), (256,), (512, 256), (512, 256), (512,), (512, 32), (32,),
              (ac * 512, 16), (ac * 16,), (mf * Ap, 64), (mf * 64,), (mf * 64, 32), (mf * 32,), (mf * 544, 256),
              (mf * 256,), (mf * 256, 16), (mf * 16,)]
    b = np.asarray(blob, dtype=np.float64)
    return [b[o:o + int(np.prod(s))].reshape(s) for o, s in zip(offsets, shapes)]


def forward(blob, offsets, V, F, A, use_mf, view, feat, prob=None):
    """view [n, ...] (V floats), feat [n, F], prob [n, A] -> (policy [n, A] clipped softmax, value [n]), float64."""
    wv, bv, we, be, wd0, wd1, bd, wp, bp, wval, bval, wep, bep, wdp, bdp, wvd, bvd, wvo, bvo = \
        blocks(blob, offsets, V, F, A, use_mf)
    relu = lambda x: np.maximum(x, 0.0)
    x = np.asarray(view, dtype=np.float64).reshape(len(view), -1)
    n = x.shape[0]
    xv = np.zeros((n, wv.shape[0]))
    xv[:, :V] = x
    f = np.zeros((n, we.shape[0]))
    f[:, :F] = feat
    concat = np.concatenate([relu(xv @ wv + bv), relu(f @ we + be)], axis=1)
    d = relu(concat @ np.concatenate([wd0, wd1], axis=1) + bd)
    logits = ((d / 0.1) @ wp + bp)[:, :A]
    e = np.exp(logits - logits.max(1, keepdims=True))
    policy = np.clip(e / e.sum(1, keepdims=True), 1e-10, 1 - 1e-10)
    if use_mf:
        p = np.zeros((n, wep.shape[0]))
        p[:, :A] = prob
        h = relu(relu(p @ wep + bep) @ wdp + bdp)
        value = (relu(np.concatenate([concat, h], axis=1) @ wvd + bvd) @ wvo + bvo)[:, 0]
    else:
        value = (d @ wval + bval)[:, 0]
    return policy, value


def mix32(h):
    h = np.asarray(h, dtype=np.uint32).copy()
    with np.errstate(over="ignore"):
        h ^= h >> _U32(16)
        h *= _U32(0x85EBCA6B)
        h ^= h >> _U32(13)
        h *= _U32(0xC2B2AE35)
        h ^= h >> _U32(16)
    return h


def uniforms(seed, step, group, rows):
    """acnet_kernels.hip ac_uniform: 24-bit float32 uniforms of rows `rows` of group `group` at step `step`."""
    with np.errstate(over="ignore"):
        a = np.array([(step * 0x9E3779B9 + group * 0x632BE5AB) & 0xFFFFFFFF], dtype=np.uint32)
        r = np.asarray(rows, dtype=np.uint32) * _U32(0x85EBCA77) + _U32(0x165667B1)
    k = _U32(seed & 0xFFFFFFFF) ^ mix32(a)[0] ^ mix32(r)
    return (mix32(k) >> _U32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def draw(policy, seed, step, group, rows):
    """The device's draw on float32 policy rows [n, A]: the first action whose running float32 sum exceeds
    u * total (total = the float32 sum in action order)."""
    p = np.asarray(policy, dtype=np.float32)
    n, A = p.shape
    tot = np.zeros(n, dtype=np.float32)
    for a in range(A):
        tot = (tot + p[:, a]).astype(np.float32)
    thr = (uniforms(seed, step, group, rows) * tot).astype(np.float32)
    run = np.zeros(n, dtype=np.float32)
    pick = np.full(n, -1, dtype=np.int64)
    for a in range(A):
        run = (run + p[:, a]).astype(np.float32)
        pick = np.where((pick < 0) & (run > thr), a, pick)
    return np.where(pick < 0, A - 1, pick).astype(np.int32)
