import os
import sys

import pytest

os.environ["OMP_NUM_THREADS"] = "1"   # the reference engine (oracle/_ref) is racy with more threads
try:        # bind every HIP user in the test process to torch's bundled HIP runtime (see magent/c_lib.py)
    import torch  # noqa: F401
except ImportError:
    pass

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd")
sys.path.insert(0, os.path.join(PKG, "python"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.append(REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")
