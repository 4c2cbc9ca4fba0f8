"""Record the reference python wrapper's ctypes call trace (build container only).

    OMP_NUM_THREADS=1 python tests/golden/make_abi_trace.py

The reference's own examples/battle_model/python/magent/gridworld.py (loaded as in
make_battle_fixtures.py) drives the reference engine (oracle/_ref) through a recording proxy of its
``_LIB``: every call is logged with the exact ctypes KIND of each argument as the wrapper passes it
(no argtypes are declared, c_lib.py:13-31): plain int, ctypes.c_int32 by value, c_void_p game
handle, bytes, c_char_p, byref(scalar), numpy-backed pointers, ctypes arrays of floats / strings /
pointers -- plus the input contents and a digest of every buffer after the call.
tests/test_abi_trace.py replays the same calls with the same kinds against any build of the ABI.

The session: the builtin battle config at 40x40, spaces / view2attack / seed, two episodes of the
reference play loop (senario_battle.play :96-171 call order; generate_map placement, rush policy),
with mean_info / global_minimap / walls / groups info and random walls in the second episode.
Output: tests/golden/abi_trace.json + abi_trace.npz (input buffers; numeric arrays only).
"""
import ctypes
import hashlib
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_battle_fixtures as mbf  # noqa: E402

SMALL = 512           # post-call buffers up to this many bytes are stored whole, larger ones as SHA-256


class _Zeros(types.ModuleType):
    """The wrapper's numpy with np.empty -> np.zeros, so the bytes a call leaves unwritten are
    deterministic (they would be allocator garbage otherwise)."""
    def __getattr__(self, name):
        return getattr(np, name)

    @staticmethod
    def empty(*a, **k):
        return np.zeros(*a, **k)


class TraceLib:
    def __init__(self, lib):
        self._lib = lib
        self.calls = []
        self.arrays = {}
        self._game = None

    def _arg(self, a, post):
        """The record of one argument; `post` collects closures that fill in its post-call state."""
        if isinstance(a, ctypes.c_void_p):
            return {"k": "game"}
        if isinstance(a, bytes):
            return {"k": "bytes", "v": a.decode("latin1")}
        if isinstance(a, int):
            return {"k": "int", "v": int(a)}
        if isinstance(a, ctypes.c_char_p):
            return {"k": "c_char_p", "v": a.value.decode("latin1")}
        if isinstance(a, ctypes.c_int32):
            return {"k": "c_int32", "v": a.value}
        if type(a).__name__ == "CArgObject":                    # ctypes.byref(x)
            obj = a._obj
            if isinstance(obj, ctypes.c_void_p):
                return {"k": "byref_void"}
            rec = {"k": "byref", "t": type(obj).__name__, "v": obj.value}
            post.append(lambda: rec.update(post=obj.value))
            return rec
        if isinstance(a, ctypes._Pointer):
            arr = getattr(a, "_arr", None)
            assert isinstance(arr, np.ndarray), "pointer without its numpy array"
            return self._array(arr, a._type_.__name__, post)
        if isinstance(a, ctypes.Array):
            et = a._type_
            if et is ctypes.c_char_p:
                return {"k": "str_array", "v": [x.decode("latin1") for x in a]}
            if et is ctypes.c_float:
                return {"k": "float_array", "v": [float(x) for x in a]}
            if issubclass(et, ctypes._Pointer):                  # (POINTER(c_float) * 2) of numpy buffers
                elems = [self._array(self._by_addr[ctypes.cast(x, ctypes.c_void_p).value], et._type_.__name__, post)
                         for x in a]
                return {"k": "ptr_array", "v": elems}
        raise TypeError("unrecorded argument kind %r" % type(a))

    def _array(self, arr, ctype, post):
        key = "a%d" % len(self.arrays)
        pre = np.ascontiguousarray(arr).copy()
        rec = {"k": "ptr", "ctype": ctype, "dtype": arr.dtype.str, "shape": list(arr.shape), "pre": None}
        if pre.nbytes <= 65536 and pre.any():
            self.arrays[key] = pre
            rec["pre"] = key
        elif pre.nbytes > 65536:
            rec["large"] = True                                   # fully written outputs (observations)

        def fix():
            b = np.ascontiguousarray(arr).tobytes()
            rec["post_sha"] = hashlib.sha256(b).hexdigest()
            if len(b) <= SMALL:
                rec["post_hex"] = b.hex()
        post.append(fix)
        return rec

    def __getattr__(self, name):
        fn = getattr(self._lib, name)

        def call(*args):
            post = []
            rec = {"fn": name, "args": [self._arg(a, post) for a in args]}
            ret = fn(*args)
            rec["ret"] = int(ret)
            for f in post:
                f()
            self.calls.append(rec)
            return ret
        return call


def main():
    assert os.environ.get("OMP_NUM_THREADS") == "1", "run with OMP_NUM_THREADS=1"
    gw, battle_cfg, scen = mbf.load_reference_magent()
    clib = sys.modules["magent.c_lib"]
    tl = TraceLib(clib._LIB)
    tl._by_addr = {}
    keep = []

    def reg(conv):
        def f(buf):
            tl._by_addr[buf.ctypes.data] = buf
            keep.append(buf)
            return conv(buf)
        return f
    # the wrapper imported these names from c_lib: route its module globals through the recorder
    gw._LIB = tl
    gw.as_float_c_array = reg(clib.as_float_c_array)
    gw.as_int32_c_array = reg(clib.as_int32_c_array)
    gw.np = _Zeros("numpy_zeros")
    import battle_driver as bd

    env = gw.GridWorld(battle_cfg.get_config(40))
    h = env.get_handles()
    for hh in h:
        env.get_view_space(hh); env.get_feature_space(hh); env.get_action_space(hh)
    attack_base, v2a = env.get_view2attack(h[0])
    env.set_seed(3)
    rng = np.random.RandomState(5)
    for ep, seed in enumerate([11, 12]):
        env.reset()
        if ep == 1:
            env.add_walls(method="random", n=30)
        import random
        random.seed(seed)
        scen.generate_map(env, 40, h)
        for t in range(24 if ep == 0 else 14):
            nums = [env.get_num(hh) for hh in h]
            obs = [env.get_observation(hh) for hh in h]
            ids = [env.get_agent_id(hh) for hh in h]
            acts = [bd.rush_policy(obs[g][0], obs[g][1], rng, v2a, attack_base, 21, eps=0.3) for g in range(2)]
            for g in range(2):
                env.set_action(h[g], acts[g])
            done = env.step()
            for g in range(2):
                env.get_reward(h[g]); env.get_alive(h[g])
            if t % 8 == 3:
                env.get_pos(h[0]); env.get_mean_info(h[1]); env.get_global_minimap(10, 10)
                env._get_groups_info(); env._get_walls_info()
            env.clear_dead()
            if done:
                break
        del nums, ids
    del env                                                       # env_delete_game (gridworld.py:631-632)
    import gc
    gc.collect()
    with open(os.path.join(HERE, "abi_trace.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_abi_trace.py",
                   "wrapper": "reference examples/battle_model/python/magent/gridworld.py",
                   "engine": "reference MAgent (oracle/_ref, OMP_NUM_THREADS=1)", "calls": tl.calls}, f,
                  separators=(",", ":"))
    np.savez_compressed(os.path.join(HERE, "abi_trace.npz"), **tl.arrays)
    print(len(tl.calls), "calls,", len(tl.arrays), "input buffers")


if __name__ == "__main__":
    main()
