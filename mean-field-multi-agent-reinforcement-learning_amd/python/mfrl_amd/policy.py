"""QNetHIP: the hand-written HIP forward (csrc/policy_kernels.hip) of the reference's Q network.

    ValueNet._construct_net  examples/battle_model/algo/base.py:123-183   -> QNetHIP.forward (q values)
    ValueNet.act             examples/battle_model/algo/base.py:228-254   -> QNetHIP.act (argmax q)

The weights come from a torch QNet (mfrl_amd.algo.nets, the layer-for-layer port that training updates):
``load(qnet)`` packs them into the device layout the kernels read -- every matrix [K][N] row-major with
the im2col / NHWC-flatten orders of TF (conv kernels [ky][kx][ci][co], Dense-Obs rows in (y, x, c) order),
K padded to a multiple of 4 with zero rows -- and uploads them in one copy.  Forward only: training keeps
the torch module (autograd); after an optimiser step call ``load`` again.

Numerics: f32 inputs and weights, f32 MFMA accumulation (one rounding per product); the result differs
from the torch module's by summation order only (|dq| ~1e-6 at these sizes, tests/test_policy_gpu.py).
"""
import ctypes

import numpy as np

import torch

from . import check, lib

_P = ctypes.c_void_p


def _ptr(t):
    return _P(t.data_ptr()) if t is not None else _P()


def rows_scratch(E, rowcap):
    """Ints of the act_rollout row-list scratch: E * rowcap rows, the row count, one total per 64-env chunk
    (include/magent_amd.h, mfx_qnet_act_rollout)."""
    return E * rowcap + 1 + (E + 63) // 64


def _stream():
    return _P(torch.cuda.current_stream().cuda_stream)


N_BLOCKS = 18      # w1 b1 w2 b2 wd bd we be wp1 bp1 wp2 bp2 w2d b2d wo bo wq bq (policy_kernels.hip)


def blob_layout(feature, n_action, use_mf):
    """(floats in the packed blob, the 18 block offsets) -- mfx_qnet_blob_size (host only, no GPU)."""
    L = lib()
    L.mfx_qnet_blob_size.restype = ctypes.c_int
    n = ctypes.c_size_t()
    off = (ctypes.c_size_t * N_BLOCKS)()
    check(L.mfx_qnet_blob_size(int(feature), int(n_action), int(bool(use_mf)), ctypes.byref(n), off),
          "mfx_qnet_blob_size")
    return n.value, list(off)


def pack_qnet(net, feature, n_action, use_mf, layout=None):
    """The device-layout blob (float32, on net's device) of a torch QNet (mfrl_amd.algo.nets.QNet)."""
    F, A, mf = int(feature), int(n_action), bool(use_mf)
    n, offsets = layout or blob_layout(F, A, mf)
    Fp, Ap = (F + 3) & ~3, (A + 3) & ~3
    dev = net.conv1.weight.device
    blob = torch.zeros(n, dtype=torch.float32, device=dev)

    def put(k, mat, rows=None, cols=None):
        m = mat.detach().to(torch.float32)
        if m.dim() == 1:
            blob[offsets[k]:offsets[k] + m.numel()] = m
            return
        R, C = m.shape
        R2, C2 = rows or R, cols or C
        full = torch.zeros((R2, C2), dtype=torch.float32, device=dev)
        full[:R, :C] = m
        blob[offsets[k]:offsets[k] + R2 * C2] = full.reshape(-1)

    put(0, net.conv1.weight.permute(2, 3, 1, 0).reshape(-1, 32), rows=64)       # [ky][kx][ci][co]
    put(1, net.conv1.bias)
    put(2, net.conv2.weight.permute(2, 3, 1, 0).reshape(-1, 32))
    put(3, net.conv2.bias)
    put(4, net.dense_obs.weight.t())                                          # [2592 (y, x, c)][256]
    put(5, net.dense_obs.bias)
    put(6, net.dense_emb.weight.t(), rows=Fp)
    put(7, net.dense_emb.bias)
    if mf:
        put(8, net.prob_emb.weight.t(), rows=Ap)
        put(9, net.prob_emb.bias)
        put(10, net.dense_act_prob.weight.t())
        put(11, net.dense_act_prob.bias)
    put(12, net.dense2.weight.t())
    put(13, net.dense2.bias)
    put(14, net.dense_out.weight.t())
    put(15, net.dense_out.bias)
    put(16, net.q_value.weight.t(), cols=32)                                  # Q columns padded to 32
    put(17, net.q_value.bias)
    return blob


class QNetHIP:
    def __init__(self, view_space, feature_space, num_actions, use_mf=False):
        h, w, c = view_space
        self.F, self.A, self.use_mf = int(feature_space[0]), int(num_actions), bool(use_mf)
        L = lib()
        for fn in ("mfx_qnet_create", "mfx_qnet_destroy", "mfx_qnet_set_weights", "mfx_qnet_forward",
                   "mfx_qnet_act_rollout"):
            getattr(L, fn).restype = ctypes.c_int
        self._L = L
        self.blob_n, self.offsets = blob_layout(self.F, self.A, self.use_mf)
        hdl = _P()
        check(L.mfx_qnet_create(int(h), int(w), int(c), self.F, self.A, int(self.use_mf), ctypes.byref(hdl)),
              "mfx_qnet_create")
        self.handle = hdl
        self._rows = None

    def __del__(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            self._L.mfx_qnet_destroy(self.handle)
            self.handle = None

    def pack(self, net):
        return pack_qnet(net, self.F, self.A, self.use_mf, (self.blob_n, self.offsets))

    def load(self, net):
        """Upload the weights of torch QNet `net` (same shapes)."""
        self._blob = self.pack(net).contiguous()
        check(self._L.mfx_qnet_set_weights(self.handle, _ptr(self._blob), ctypes.c_size_t(self.blob_n), _stream()),
              "mfx_qnet_set_weights")
        return self

    # ------------------------------------------------------------------ forward
    def forward(self, view, feature, prob=None, want_q=True):
        """view [n, 13, 13, 7], feature [n, F], prob [n, A] (mean field) float32 CUDA tensors ->
        (q [n, A] float32 or None, actions [n] int32 = argmax q)."""
        n = view.shape[0]
        view = view.reshape(n, -1).contiguous().float()
        feature = feature.reshape(n, -1).contiguous().float()
        if self.use_mf:
            assert prob is not None and prob.shape[0] == n
            prob = prob.reshape(n, -1).contiguous().float()
        q = torch.empty((n, self.A), dtype=torch.float32, device=view.device) if want_q else None
        act = torch.empty(n, dtype=torch.int32, device=view.device)
        check(self._L.mfx_qnet_forward(self.handle, _ptr(view), _ptr(feature), _ptr(prob if self.use_mf else None),
                                       int(n), _ptr(q), _ptr(act), _stream()), "mfx_qnet_forward")
        return q, act

    def act(self, view, feature, prob=None):
        return self.forward(view, feature, prob, want_q=False)[1]

    def act_rollout(self, eng, group):
        """Actions of group `group` of a BattleBatch rollout from its current observation buffers and
        former mean actions, written into the rollout's action buffer [E][G][rowcap] (live rows only)."""
        E, rc, G = eng.n_envs, eng.rowcap, len(eng.handles)
        if self._rows is None or self._rows.numel() < rows_scratch(E, rc):
            self._rows = torch.empty(rows_scratch(E, rc), dtype=torch.int32, device="cuda")
        ptr = {}
        for name in ("view", "feature", "group_num", "mean_action", "actions"):
            p, nb = _P(), ctypes.c_size_t()
            eng._check(eng._dll.mfx_battle_rollout_buffer(eng.game, name.encode(), group if name in ("view", "feature")
                                                          else 0, ctypes.byref(p), ctypes.byref(nb)), "rollout_buffer")
            ptr[name] = p
        stride = eng.mean_stride()
        check(self._L.mfx_qnet_act_rollout(self.handle, ptr["view"], ptr["feature"], ptr["group_num"],
                                           ptr["mean_action"], int(stride), int(E), int(G), int(group), int(rc),
                                           _P(self._rows.data_ptr()), _P(self._rows.data_ptr() + 4 * E * rc),
                                           ptr["actions"], _P(eng.stream_handle())), "mfx_qnet_act_rollout")


# ---------------------------------------------------------------------------------------------------------------
# the actor-critic network (ActorCritic / MFAC, algo/ac.py:48-98, :219-276) on csrc/acnet_kernels.hip
# ---------------------------------------------------------------------------------------------------------------
AC_BLOCKS = 19     # wv bv we be wd0 wd1 bd wp bp wval bval wep bep wdp bdp wvd bvd wvo bvo (acnet_kernels.hip)


def acnet_layout(view_floats, feature, n_action, use_mf):
    """(floats in the packed blob, the 19 block offsets) -- mfx_acnet_blob_size (host only, no GPU)."""
    L = lib()
    L.mfx_acnet_blob_size.restype = ctypes.c_int
    n = ctypes.c_size_t()
    off = (ctypes.c_size_t * AC_BLOCKS)()
    check(L.mfx_acnet_blob_size(int(view_floats), int(feature), int(n_action), int(bool(use_mf)), ctypes.byref(n), off),
          "mfx_acnet_blob_size")
    return n.value, list(off)


def pack_acnet(net, view_floats, feature, n_action, use_mf, layout=None):
    """The device-layout blob (float32, on net's device) of a torch ACNet (mfrl_amd.algo.nets.ACNet)."""
    V, F, A, mf = int(view_floats), int(feature), int(n_action), bool(use_mf)
    n, offsets = layout or acnet_layout(V, F, A, mf)
    Vp, Fp, Ap = (V + 3) & ~3, (F + 3) & ~3, (A + 3) & ~3
    dev = net.h_view.weight.device
    blob = torch.zeros(n, dtype=torch.float32, device=dev)

    def put(k, mat, rows=None, cols=None):
        m = mat.detach().to(torch.float32)
        if m.dim() == 1:
            blob[offsets[k]:offsets[k] + m.numel()] = m
            return
        R, C = m.shape
        full = torch.zeros((rows or R, cols or C), dtype=torch.float32, device=dev)
        full[:R, :C] = m
        blob[offsets[k]:offsets[k] + full.numel()] = full.reshape(-1)

    put(0, net.h_view.weight.t(), rows=Vp)                    # [V (NHWC flatten)][256]
    put(1, net.h_view.bias)
    put(2, net.h_emb.weight.t(), rows=Fp)
    put(3, net.h_emb.bias)
    wd = net.dense.weight.t()                                 # [512 in][512 out], by output halves
    put(4, wd[:, :256])
    put(5, wd[:, 256:])
    put(6, net.dense.bias)
    put(7, net.policy.weight.t(), cols=32)
    put(8, net.policy.bias)
    if mf:
        put(11, net.emb_prob.weight.t(), rows=Ap)
        put(12, net.emb_prob.bias)
        put(13, net.dense_prob.weight.t())
        put(14, net.dense_prob.bias)
        put(15, net.value_dense.weight.t())                   # [544 = concat 512 + dense_prob 32][256]
        put(16, net.value_dense.bias)
        put(17, net.value.weight.t(), cols=16)
        put(18, net.value.bias)
    else:
        put(9, net.value.weight.t(), cols=16)
        put(10, net.value.bias)
    return blob


class ACNetHIP:
    """Forward of ActorCritic / MFAC on the HIP kernel k_acnet: the clipped softmax policy, the value, and the
    draw of tf.multinomial(log(policy)) from a counter-hash uniform (seed, step, group, row)."""

    def __init__(self, view_space, feature_space, num_actions, use_mf=False):
        V = 1
        for d in view_space:
            V *= int(d)
        self.V, self.F, self.A, self.use_mf = V, int(feature_space[0]), int(num_actions), bool(use_mf)
        L = lib()
        for fn in ("mfx_acnet_create", "mfx_acnet_destroy", "mfx_acnet_set_weights", "mfx_acnet_forward",
                   "mfx_acnet_act_rollout", "mfx_acnet_set_input_support", "mfx_acnet_input_support_size"):
            getattr(L, fn).restype = ctypes.c_int
        self._L = L
        self.blob_n, self.offsets = acnet_layout(self.V, self.F, self.A, self.use_mf)
        hdl = _P()
        check(L.mfx_acnet_create(self.V, self.F, self.A, int(self.use_mf), ctypes.byref(hdl)), "mfx_acnet_create")
        self.handle = hdl
        self._rows = {}
        self._support = None

    def __del__(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            self._L.mfx_acnet_destroy(self.handle)
            self.handle = None

    def pack(self, net):
        return pack_acnet(net, self.V, self.F, self.A, self.use_mf, (self.blob_n, self.offsets))

    def load(self, net):
        """Upload the weights of torch ACNet `net` (same shapes)."""
        self._blob = self.pack(net).contiguous()
        check(self._L.mfx_acnet_set_weights(self.handle, _ptr(self._blob), ctypes.c_size_t(self.blob_n), _stream()),
              "mfx_acnet_set_weights")
        return self

    def set_input_support(self, mask):
        """mask: uint8/bool [V], 1 where the view can be non-zero (e.g. BattleBatch.view_support), or None for the
        dense order.  Later forwards run the view layer over the supported inputs only -- the same results bit for
        bit while the view is zero elsewhere, which the caller guarantees (the engine's observation buffers are)."""
        if mask is None:
            check(self._L.mfx_acnet_set_input_support(self.handle, None, 0, _stream()), "mfx_acnet_set_input_support")
            self._support = None
            return self
        m = np.ascontiguousarray(np.asarray(mask, dtype=np.uint8).reshape(-1))
        check(self._L.mfx_acnet_set_input_support(self.handle, m.ctypes.data_as(ctypes.c_void_p), int(m.size),
                                                  _stream()), "mfx_acnet_set_input_support")
        self._support = m.copy()
        return self

    def input_support_size(self):
        """Inputs the view layer runs over (0: the dense order)."""
        k = ctypes.c_int()
        check(self._L.mfx_acnet_input_support_size(self.handle, ctypes.byref(k)), "mfx_acnet_input_support_size")
        return k.value

    def forward(self, view, feature, prob=None, want_policy=True, want_value=False, want_act=True, seed=0, step=0):
        """view [n, ...] (flattened to V), feature [n, F], prob [n, A] (the MF value head) float32 CUDA tensors
        -> (policy [n, A] or None, value [n] or None, actions [n] int32 or None; row i drawn with (seed, step,
        group 0, row i))."""
        n = view.shape[0]
        view = view.reshape(n, -1).contiguous().float()
        feature = feature.reshape(n, -1).contiguous().float()
        if want_value and self.use_mf:
            assert prob is not None and prob.shape[0] == n
            prob = prob.reshape(n, -1).contiguous().float()
        else:
            prob = None
        dev = view.device
        pol = torch.empty((n, self.A), dtype=torch.float32, device=dev) if want_policy else None
        val = torch.empty(n, dtype=torch.float32, device=dev) if want_value else None
        act = torch.empty(n, dtype=torch.int32, device=dev) if want_act else None
        check(self._L.mfx_acnet_forward(self.handle, _ptr(view), _ptr(feature), _ptr(prob), int(n), _ptr(pol), _ptr(val),
                                        _ptr(act), ctypes.c_uint32(seed & 0xFFFFFFFF), ctypes.c_uint32(step & 0xFFFFFFFF),
                                        _stream()), "mfx_acnet_forward")
        return pol, val, act

    def act(self, view, feature, seed=0, step=0):
        return self.forward(view, feature, want_policy=False, seed=seed, step=step)[2]

    def act_rollout(self, eng, group, seed, step, support=True):
        """Sampled actions of group `group` of a BattleBatch rollout from its current observation buffers,
        written into the rollout's action buffer [E][G][rowcap] (live rows; row j of env e drawn with (seed,
        step, group, e * rowcap + j)).  Nothing is read back to the host.  support: run the view layer over the
        inputs the engine's view can make non-zero only (BattleBatch.view_support; bit-identical).  The row-list
        scratch is per engine, so engines on different streams may share this network."""
        E, rc, G = eng.n_envs, eng.rowcap, len(eng.handles)
        if support:
            m = eng.view_support(group)
            if self._support is None or not np.array_equal(self._support, m):
                self.set_input_support(m)
        elif self._support is not None:
            self.set_input_support(None)
        rows = self._rows.get(id(eng))
        if rows is None or rows.numel() < rows_scratch(E, rc):
            rows = self._rows[id(eng)] = torch.empty(rows_scratch(E, rc), dtype=torch.int32, device="cuda")
        ptr = {}
        for name in ("view", "feature", "group_num", "actions"):
            p, nb = _P(), ctypes.c_size_t()
            eng._check(eng._dll.mfx_battle_rollout_buffer(eng.game, name.encode(), group if name in ("view", "feature")
                                                          else 0, ctypes.byref(p), ctypes.byref(nb)), "rollout_buffer")
            ptr[name] = p
        check(self._L.mfx_acnet_act_rollout(self.handle, ptr["view"], ptr["feature"], ptr["group_num"], int(E), int(G),
                                            int(group), int(rc), _P(rows.data_ptr()),
                                            _P(rows.data_ptr() + 4 * E * rc), ptr["actions"],
                                            ctypes.c_uint32(seed & 0xFFFFFFFF), ctypes.c_uint32(step & 0xFFFFFFFF),
                                            _P(eng.stream_handle())), "mfx_acnet_act_rollout")
