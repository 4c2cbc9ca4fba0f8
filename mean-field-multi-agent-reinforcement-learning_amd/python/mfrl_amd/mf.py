"""Mean-field pieces of the training loop on device (torch tensors in, torch tensors out).

    mean_action(actions, counts, n_action)   senario_battle.py:141 (former_act_prob), float64
    mfq_target(e_q, t_q, rewards, dones, g)  algo/base.py:192-220 (ValueNet.calc_target_q), float64
    mfac_returns(rewards, offsets, values, g) algo/ac.py:305-320 (discounted returns, float64 running
                                             return stored as float32: the reference's NumPy-1 rules)
"""
import ctypes

import torch

from . import check, lib


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def mean_action(actions, counts, n_action):
    """actions int32 [B, rowcap] (rows past counts[b] ignored), counts int32 [B] -> float64 [B, n_action]."""
    B, rowcap = actions.shape
    out = torch.empty((B, n_action), dtype=torch.float64, device=actions.device)
    L = lib()
    L.mfx_mean_action.restype = ctypes.c_int
    check(L.mfx_mean_action(_p(actions.contiguous()), _p(counts.contiguous()), B, rowcap, n_action, _p(out),
                            _stream()), "mfx_mean_action")
    return out


def mfq_target(e_q, t_q, rewards, dones, gamma=0.95):
    """target = r + (1 - done) * t_q[argmax e_q] * gamma, float64 [M] (dones: bool/uint8 [M])."""
    M, A = e_q.shape
    out = torch.empty(M, dtype=torch.float64, device=e_q.device)
    d = dones.to(torch.uint8).contiguous()
    L = lib()
    L.mfx_mfq_target.restype = ctypes.c_int
    check(L.mfx_mfq_target(_p(e_q.contiguous()), _p(t_q.contiguous()), _p(rewards.contiguous()), _p(d), M, A,
                           ctypes.c_double(gamma), _p(out), _stream()), "mfx_mfq_target")
    return out


def mfac_returns(rewards, offsets, values, gamma=0.95, numpy1=True):
    """Per-episode discounted returns, in place on float32 rewards; offsets int64 [E+1].

    numpy1: the promotion of the reference's NumPy-1 era (keep in float64); False: NEP 50 (float32)."""
    L = lib()
    L.mfx_mfac_returns.restype = ctypes.c_int
    check(L.mfx_mfac_returns(_p(rewards), _p(offsets.contiguous()), _p(values.contiguous()), len(values),
                             ctypes.c_double(gamma), int(bool(numpy1)), _stream()), "mfx_mfac_returns")
    return rewards
