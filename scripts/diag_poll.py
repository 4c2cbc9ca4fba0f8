"""Diagnostic: the signalling floor of a resident one-wave server inside this process (torch's HIP
runtime), from libmagent.so's mfx_diag_poll_rtt; compare with scripts/micro/poll_rtt (plain HIP)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
import torch  # noqa: E402,F401
import magent  # noqa: E402

lib = magent.load_library(None).dll
fn = lib.mfx_diag_poll_rtt
fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
for fence in (0, 1, 0):
    us = ctypes.c_double()
    rc = fn(20000, fence, ctypes.byref(us))
    print("in-process poll round trip, fence=%d: rc %d, %.2f us" % (fence, rc, us.value))
