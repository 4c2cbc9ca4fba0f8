"""`from examples.battle_model.algo import spawn_ai, tools` -> mfrl_amd.algo (PyTorch-ROCm)."""
from mfrl_amd.algo import AC, IL, MFAC, MFQ, ac, q_learning, spawn_ai, tools  # noqa: F401
