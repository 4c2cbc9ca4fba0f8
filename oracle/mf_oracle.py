"""TEST ORACLE ONLY -- the mean-field training-loop expressions, restated from the reference's source
text in numpy (tests may use it; the product never does).

* mean_action  -- senario_battle.py:141, the reference expression verbatim in meaning.  Pinned:
                  tests/golden/battle_*.npz hold its value on every recorded step.
* mfq_target   -- algo/base.py:208-220 (ValueNet.calc_target_q after the TF session call).
* mfac_returns -- algo/ac.py:305-320 (MFAC.train's backward return loop).
  Both PINNED: tests/golden/algo_mfq_target.npz and algo_mfac_returns.npz hold the outputs of the
  reference's own lines, run here under a tensorflow stub (tests/golden/make_algo_fixtures.py).
  mfac_returns has two promotion rules: numpy1 (the reference's TF1-era NumPy: np.float32 * python
  float is float64, so keep accumulates in float64) and nep50 (NumPy 2: float32 throughout).
"""
import numpy as np


def mean_action(acts, n_action):
    return np.mean(list(map(lambda x: np.eye(n_action)[x], acts)), axis=0, keepdims=True)


def mfq_target(e_q, t_q, rewards, dones, gamma=0.95):
    act_idx = np.argmax(e_q, axis=1)
    q_values = t_q[np.arange(len(t_q)), act_idx]
    return rewards + (1. - dones) * q_values.reshape(-1) * gamma


def mfac_returns(rewards, value, gamma=0.95, numpy1=True):
    r = np.array(rewards, dtype=np.float32)
    # NumPy 1: keep * gamma promotes the float32 scalar to float64 (exact), and it stays float64
    keep = np.float64(np.float32(value)) if numpy1 else np.float32(value)
    for i in reversed(range(len(r))):
        keep = keep * gamma + r[i]
        r[i] = keep
    return r
