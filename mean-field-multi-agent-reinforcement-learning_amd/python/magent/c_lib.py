"""Binding of the engine's C ABI (reference python/magent/c_lib.py:13-55).

The library is located like the reference does it -- ``<package>/../../build/libmagent.so``
-- unless ``MAGENT_LIB`` names another build.  Because the ABI is the reference's own
(runtime_api.h:20-55), the same binding also drives the reference engine build and the
C oracle used by the tests (``load_library(path)``).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB = os.path.normpath(os.path.join(_HERE, "..", "..", "build", "libmagent.so"))

_c = ctypes
_SIGS = {
    "env_new_game": [_c.POINTER(_c.c_void_p), _c.c_char_p],
    "env_delete_game": [_c.c_void_p],
    "env_config_game": [_c.c_void_p, _c.c_char_p, _c.c_void_p],
    "env_reset": [_c.c_void_p],
    "env_get_observation": [_c.c_void_p, _c.c_int, _c.POINTER(_c.POINTER(_c.c_float))],
    "env_set_action": [_c.c_void_p, _c.c_int, _c.POINTER(_c.c_int32)],
    "env_step": [_c.c_void_p, _c.POINTER(_c.c_int32)],
    "env_get_reward": [_c.c_void_p, _c.c_int, _c.POINTER(_c.c_float)],
    "env_get_info": [_c.c_void_p, _c.c_int, _c.c_char_p, _c.c_void_p],
    "env_render": [_c.c_void_p],
    "gridworld_register_agent_type": [_c.c_void_p, _c.c_char_p, _c.c_int, _c.POINTER(_c.c_char_p),
                                      _c.POINTER(_c.c_float)],
    "gridworld_new_group": [_c.c_void_p, _c.c_char_p, _c.POINTER(_c.c_int32)],
    "gridworld_add_agents": [_c.c_void_p, _c.c_int, _c.c_int, _c.c_char_p, _c.POINTER(_c.c_int32),
                             _c.POINTER(_c.c_int32), _c.POINTER(_c.c_int32)],
    "gridworld_clear_dead": [_c.c_void_p],
    "gridworld_define_agent_symbol": [_c.c_void_p, _c.c_int, _c.c_int, _c.c_int],
    "gridworld_define_event_node": [_c.c_void_p, _c.c_int, _c.c_int, _c.POINTER(_c.c_int32), _c.c_int],
    "gridworld_add_reward_rule": [_c.c_void_p, _c.c_int, _c.POINTER(_c.c_int32), _c.POINTER(_c.c_float),
                                  _c.c_int, _c.c_bool, _c.c_bool],
}


class EngineError(RuntimeError):
    pass


def _pin_hip_runtime():
    """PyTorch-ROCm wheels bundle their own HIP/HSA runtime (SONAME libamdhip64.so.7).  If the
    engine were loaded first it would pull /opt/rocm's runtime into the process, and a later
    `import torch` would bring a second, conflicting HSA runtime ("No HIP GPUs are available").
    Importing torch first makes the engine bind to torch's runtime.  MAGENT_PIN_TORCH=0 skips it
    (processes that never use torch)."""
    if os.environ.get("MAGENT_PIN_TORCH", "1") == "0":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


class Library:
    """A loaded engine library with checked calls (``lib.env_step(...)`` raises on failure)."""

    def __init__(self, path):
        self.path = path
        if "amd" in os.path.basename(os.path.dirname(os.path.dirname(path))) or path == DEFAULT_LIB:
            _pin_hip_runtime()
        self._dll = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        for name, argtypes in _SIGS.items():
            fn = getattr(self._dll, name)
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int
        self._last_error = getattr(self._dll, "mfx_last_error", None)
        if self._last_error is not None:
            self._last_error.restype = ctypes.c_char_p

    @property
    def dll(self):
        return self._dll

    def __getattr__(self, name):
        fn = getattr(self._dll, name)

        def checked(*args):
            ret = fn(*args)
            if ret != 0:
                msg = self._last_error().decode() if self._last_error is not None else ""
                raise EngineError("%s failed (%d): %s" % (name, ret, msg))
            return ret
        checked.__name__ = name
        setattr(self, name, checked)         # made once per function: later calls skip __getattr__
        return checked


_LIB = None


def load_library(path=None):
    return Library(path or os.environ.get("MAGENT_LIB") or DEFAULT_LIB)


def get_lib():
    """The process-wide default engine (the HIP build unless MAGENT_LIB says otherwise)."""
    global _LIB
    if _LIB is None:
        path = os.environ.get("MAGENT_LIB") or DEFAULT_LIB
        if not os.path.exists(path):
            raise EngineError("engine library not found at %s -- build it with `make` in the package "
                              "directory (or __graft_entry__.build())" % path)
        _LIB = Library(path)
    return _LIB


def as_float_c_array(buf):
    return buf.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def as_int32_c_array(buf):
    return buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def as_bool_c_array(buf):
    return buf.ctypes.data_as(ctypes.POINTER(ctypes.c_bool))
