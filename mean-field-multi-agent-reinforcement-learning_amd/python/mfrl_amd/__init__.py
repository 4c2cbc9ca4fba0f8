"""mfrl_amd: the batched, device-resident API of the MI355X Battle / Ising engine.

    magent            drop-in of the reference python package (one env, host buffers)
    mfrl_amd.battle   BattleBatch: E envs in HBM, fused rollout step (bench path)
    mfrl_amd.ising    Ising lattice + tabular MF-Q (main_MFQ_Ising.py) on device
    mfrl_amd.mf       mean-action pooling, MF-Q target, MF-AC discounted returns
"""
import ctypes
import os

from magent.c_lib import DEFAULT_LIB, EngineError, _pin_hip_runtime

_DLL = None


def lib():
    """The engine library (ctypes.CDLL) with the mfx_* batched entry points."""
    global _DLL
    if _DLL is None:
        path = os.environ.get("MAGENT_LIB") or DEFAULT_LIB
        if not os.path.exists(path):
            raise EngineError("engine library not found at %s (run `make` in the package dir)" % path)
        _pin_hip_runtime()
        _DLL = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        _DLL.mfx_last_error.restype = ctypes.c_char_p
        _DLL.mfx_build_info.restype = ctypes.c_char_p
    return _DLL


def check(ret, what=""):
    if ret != 0:
        raise EngineError("%s failed: %s" % (what, lib().mfx_last_error().decode()))
    return ret
