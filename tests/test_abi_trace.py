"""The reference python wrapper's own ctypes calls, replayed against a build of the ABI.

tests/golden/abi_trace.json records every call the reference examples/battle_model/python/magent/
gridworld.py made into the reference engine over a two-episode session (make_abi_trace.py): the
exact ctypes kind of every argument (no argtypes are declared, c_lib.py:13-31 -- plain int, c_int32
by value, c_void_p handle, bytes, c_char_p, byref(scalar), numpy-backed pointers, ctypes arrays),
the input buffers and the digest of every buffer after the call.  Replaying it with the same kinds
shows the wrapper binds a library unchanged: every return code and every output byte must match.

CPU: the replayer against the reference build itself (oracle/_ref), when present.
GPU: libmagent.so, with the drop-in's one-launch step and with the per-call path."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import common

TRACE = os.path.join(common.GOLDEN, "abi_trace.json")
BUFS = os.path.join(common.GOLDEN, "abi_trace.npz")


def replay(lib_path, limit=None):
    if os.path.abspath(lib_path) == os.path.abspath(common.REF_LIB):
        common.pin_ref_threads()
    lib = ctypes.CDLL(lib_path, ctypes.RTLD_GLOBAL)      # as c_lib.py:30 loads it: no argtypes, no restype
    calls = json.load(open(TRACE))["calls"]
    pre = np.load(BUFS)
    game = ctypes.c_void_p()
    problems = []

    def buffer(d, keep, outs):
        arr = pre[d["pre"]].copy() if d.get("pre") else np.zeros(d["shape"], dtype=np.dtype(d["dtype"]))
        keep.append(arr)
        outs.append((d, arr))
        return arr.ctypes.data_as(ctypes.POINTER(getattr(ctypes, d["ctype"])))

    for i, c in enumerate(calls[:limit]):
        args, keep, outs = [], [], []
        for d in c["args"]:
            k = d["k"]
            if k == "game":
                args.append(game)
            elif k == "bytes":
                args.append(d["v"].encode("latin1"))
            elif k == "int":
                args.append(d["v"])
            elif k == "c_char_p":
                args.append(ctypes.c_char_p(d["v"].encode("latin1")))
            elif k == "c_int32":
                args.append(ctypes.c_int32(d["v"]))
            elif k == "byref_void":
                args.append(ctypes.byref(game))
            elif k == "byref":
                obj = getattr(ctypes, d["t"])(d["v"])
                keep.append(obj)
                outs.append((d, obj))
                args.append(ctypes.byref(obj))
            elif k == "ptr":
                args.append(buffer(d, keep, outs))
            elif k == "str_array":
                a = (ctypes.c_char_p * len(d["v"]))(*[x.encode("latin1") for x in d["v"]])
                keep.append(a)
                args.append(a)
            elif k == "float_array":
                a = (ctypes.c_float * len(d["v"]))(*d["v"])
                keep.append(a)
                args.append(a)
            elif k == "ptr_array":
                et = ctypes.POINTER(getattr(ctypes, d["v"][0]["ctype"]))
                a = (et * len(d["v"]))()
                for j, e in enumerate(d["v"]):
                    a[j] = buffer(e, keep, outs)
                keep.append(a)
                args.append(a)
            else:
                raise AssertionError("unknown argument kind %s" % k)
        ret = getattr(lib, c["fn"])(*args)
        if ret != c["ret"]:
            problems.append("call %d %s: returned %d, reference %d" % (i, c["fn"], ret, c["ret"]))
        for d, o in outs:
            if d["k"] == "byref":
                if o.value != d["post"]:
                    problems.append("call %d %s: output %r, reference %r" % (i, c["fn"], o.value, d["post"]))
            elif hashlib.sha256(np.ascontiguousarray(o).tobytes()).hexdigest() != d["post_sha"]:
                problems.append("call %d %s: buffer %s differs" % (i, c["fn"], d["shape"]))
        if len(problems) > 5:
            break
    return problems


def test_trace_covers_the_wrapper_surface():
    calls = json.load(open(TRACE))["calls"]
    fns = {c["fn"] for c in calls}
    for fn in ("env_new_game", "env_config_game", "gridworld_register_agent_type", "gridworld_new_group",
               "gridworld_define_agent_symbol", "gridworld_define_event_node", "gridworld_add_reward_rule",
               "env_reset", "gridworld_add_agents", "env_get_observation", "env_set_action", "env_step",
               "env_get_reward", "env_get_info", "gridworld_clear_dead", "env_delete_game"):
        assert fn in fns, fn
    kinds = {d["k"] for c in calls for d in c["args"]}
    assert {"game", "bytes", "int", "c_int32", "byref", "byref_void", "ptr", "str_array", "float_array",
            "ptr_array"} <= kinds
    # the wrapper's 6-argument call of the 7-parameter add_reward_rule (gridworld.py:719-722)
    assert all(len(c["args"]) == 6 for c in calls if c["fn"] == "gridworld_add_reward_rule")


def test_replayer_reproduces_the_reference_build():
    if not os.path.exists(common.REF_LIB):
        pytest.skip("oracle/_ref not built (build container only)")
    assert replay(common.REF_LIB) == []


@pytest.mark.gpu
@pytest.mark.parametrize("fast", ["1", "0"])
def test_reference_wrapper_calls_bind_libmagent(fast, monkeypatch):
    monkeypatch.setenv("MFX_DROPIN_FAST", fast)
    assert replay(common.HIP_LIB) == []
