"""BattleBatch: E independent Battle envs resident in HBM (include/magent_amd.h, mfx_battle_*).

The configuration path is the reference's own (magent.GridWorld serialises the config
through the env_*/gridworld_* ABI); then the env is switched to E instances before its
first reset.  Two ways to step it:

* per call, on device buffers (``observe / set_action / step / get / clear_dead``) -- the
  reference call sequence, batched;
* fused (``rollout_init / rollout_step``) -- one kernel launch per training-loop step
  (obs x G, on-device rush policy, set_action, step, reward, mean action, clear_dead,
  episode restart) for all envs: the throughput path measured by bench.py.
"""
import ctypes

import numpy as np

import magent
from magent.gridworld import GridWorld

from . import check, lib

GET_NUM, GET_REWARD, GET_ID, GET_ALIVE, GET_POS, GET_HP = range(6)


class BattleBatch:
    def __init__(self, map_size, n_envs, config="battle", stream=None):
        L = magent.load_library(lib()._name)
        self.env = GridWorld(config, map_size=map_size, lib=L) if isinstance(config, str) else GridWorld(config, lib=L)
        self._dll = L.dll
        for fn in ("mfx_battle_set_num_envs", "mfx_battle_set_stream", "mfx_battle_observe",
                   "mfx_battle_set_action", "mfx_battle_step", "mfx_battle_get", "mfx_battle_clear_dead",
                   "mfx_battle_sync", "mfx_battle_rollout_init", "mfx_battle_rollout_step",
                   "mfx_battle_rollout_buffer", "mfx_battle_rollout_copy", "mfx_battle_rollout_rowcap",
                   "mfx_battle_rollout_info", "mfx_battle_group_capacity", "mfx_battle_rollout_set_substeps",
                   "mfx_battle_rollout_copy_at", "mfx_battle_rollout_check", "mfx_battle_rollout_path",
                   "mfx_battle_rollout_policy_step", "mfx_battle_rollout_sum_lanes", "mfx_battle_rollout_mean_stride",
                   "mfx_battle_rollout_get_substeps"):
            try:
                getattr(self._dll, fn).restype = ctypes.c_int
            except AttributeError:          # an older build of the library (A/B runs)
                pass
        self._dll.mfx_last_error.restype = ctypes.c_char_p
        self.handles = self.env.get_handles()
        self.n_envs = n_envs
        self.game = self.env.game
        self._check(self._dll.mfx_battle_set_num_envs(self.game, n_envs), "set_num_envs")
        if stream is not None:
            self.set_stream(stream)

    def _check(self, ret, what):
        if ret != 0:
            raise magent.EngineError("%s failed: %s" % (what, self._dll.mfx_last_error().decode()))

    def set_stream(self, stream):
        """stream: a torch.cuda.Stream (or a raw hipStream_t as int)."""
        raw = getattr(stream, "cuda_stream", stream)
        self._check(self._dll.mfx_battle_set_stream(self.game, ctypes.c_void_p(raw)), "set_stream")
        self._stream_raw = raw

    def stream_handle(self):
        """The hipStream_t the engine launches on (0: the null stream)."""
        return getattr(self, "_stream_raw", 0) or 0

    # ------------------------------------------------------------------ reference call sequence
    def reset(self):
        self.env.reset()

    def add_agents(self, group, pos):
        self.env.add_agents(self.handles[group], method="custom", pos=pos)

    def capacity(self, group):
        c = ctypes.c_int()
        self._check(self._dll.mfx_battle_group_capacity(self.game, group, ctypes.byref(c)), "capacity")
        return c.value

    def observe(self, group, view, feature, rowcap):
        self._check(self._dll.mfx_battle_observe(self.game, group, ctypes.c_void_p(view.data_ptr()),
                                                 ctypes.c_void_p(feature.data_ptr()), rowcap), "observe")

    def set_action(self, group, actions, rowcap):
        self._check(self._dll.mfx_battle_set_action(self.game, group, ctypes.c_void_p(actions.data_ptr()), rowcap),
                    "set_action")

    def step(self, done=None):
        ptr = ctypes.c_void_p(done.data_ptr()) if done is not None else ctypes.c_void_p()
        self._check(self._dll.mfx_battle_step(self.game, ptr), "step")

    def get(self, group, what, out, rowcap):
        self._check(self._dll.mfx_battle_get(self.game, group, what, ctypes.c_void_p(out.data_ptr()), rowcap), "get")

    def clear_dead(self):
        self._check(self._dll.mfx_battle_clear_dead(self.game), "clear_dead")

    def sync(self):
        self._check(self._dll.mfx_battle_sync(self.game), "sync")

    # ------------------------------------------------------------------ fused rollout
    def rollout_init(self, placement, max_steps=400, eps=0.2, seed=0, stagger=True):
        """placement: list over groups of [(x, y[, dir]), ...] re-applied at every episode start.

        stagger: spread the episode phase over envs (env e's first episode is cut short by
        e*max_steps/E steps), so after max_steps steps the batch holds every phase of an episode."""
        G = len(self.handles)
        n = (ctypes.c_int * G)(*[len(p) for p in placement])
        self._keep = [np.ascontiguousarray(np.asarray(p, dtype=np.int32)[:, :2]) for p in placement]
        xs = [np.ascontiguousarray(a[:, 0]) for a in self._keep]
        ys = [np.ascontiguousarray(a[:, 1]) for a in self._keep]
        self._keep += xs + ys
        P = ctypes.POINTER(ctypes.c_int)
        px = (P * G)(*[a.ctypes.data_as(P) for a in xs])
        py = (P * G)(*[a.ctypes.data_as(P) for a in ys])
        self._check(self._dll.mfx_battle_rollout_init(self.game, n, px, py, max_steps, ctypes.c_float(eps),
                                                      ctypes.c_uint(seed), int(stagger)),
                    "rollout_init")
        rc = ctypes.c_int()
        self._dll.mfx_battle_rollout_rowcap(self.game, ctypes.byref(rc))
        self.rowcap = rc.value

    def rollout_info(self):
        """(persistent grid in workgroups, dynamic LDS bytes per workgroup) of the fused rollout."""
        g, b = ctypes.c_int(), ctypes.c_int()
        self._check(self._dll.mfx_battle_rollout_info(self.game, ctypes.byref(g), ctypes.byref(b)), "rollout_info")
        return g.value, b.value

    def rollout_check(self):
        """Synchronise; raise on a device error word or an error of the large-env queue kernel
        (k_rollout_bigq: a stall, a workgroup outside XCDs 0-7, the hand-off guard)."""
        self._check(self._dll.mfx_battle_rollout_check(self.game), "rollout_check")

    PATHS = ("k_rollout", "k_rollout_obs+k_rollout", "k_observe_items+k_rollout_big", "k_rollout_bigq")

    def rollout_path(self):
        """Name of the kernels rollout_step runs (the path rollout_init / the last re-plan chose)."""
        p = ctypes.c_int()
        self._check(self._dll.mfx_battle_rollout_path(self.game, ctypes.byref(p)), "rollout_path")
        return self.PATHS[p.value]

    def rollout_sum_lanes(self, n_agents):
        """Lanes over which the rollout sums a group's rewards of an env with n_agents agents (the order
        of the episode-return sums; the oracle replay restates it)."""
        p = ctypes.c_int()
        self._check(self._dll.mfx_battle_rollout_sum_lanes(self.game, int(n_agents), ctypes.byref(p)),
                    "rollout_sum_lanes")
        return p.value

    def rollout_substeps(self, n_sub):
        """Consecutive steps of every env per k_rollout launch (results do not depend on it); 0: the engine
        picks per path and batch size (get_substeps reports it)."""
        self._check(self._dll.mfx_battle_rollout_set_substeps(self.game, int(n_sub)), "rollout_set_substeps")

    def get_substeps(self):
        """Steps per launch in force (after rollout_init)."""
        p = ctypes.c_int()
        self._check(self._dll.mfx_battle_rollout_get_substeps(self.game, ctypes.byref(p)), "rollout_get_substeps")
        return p.value

    def rollout_step(self, n_steps=1):
        self._check(self._dll.mfx_battle_rollout_step(self.game, n_steps), "rollout_step")

    # ------------------------------------------------------------------ learned policy in the loop
    def rollout_policy_observe(self):
        """Write every env's observation into the rollout buffers (the first step of a learned-policy loop)."""
        self._check(self._dll.mfx_battle_rollout_policy_step(self.game, 2), "rollout_policy_step")

    def rollout_policy_step(self):
        """Act with the rollout's action buffer (a policy's forward on the current observation, e.g.
        mfrl_amd.policy.QNetHIP.act_rollout), step every env, observe the new state."""
        self._check(self._dll.mfx_battle_rollout_policy_step(self.game, 1), "rollout_policy_step")

    def mean_stride(self):
        """Doubles per [env][group] row of the mean-action buffer (the largest n_action), as the engine laid
        it out (the buffer itself may be larger: device buffers are kept across re-initialisations)."""
        p = ctypes.c_int()
        self._check(self._dll.mfx_battle_rollout_mean_stride(self.game, ctypes.byref(p)), "rollout_mean_stride")
        return p.value

    STORE_SHAPES = tuple("%s per workgroup, %s%s" % (c, g, nt) for c, g in (
        ("4 KiB", "one workgroup per chunk"), ("8 KiB", "one workgroup per chunk"), ("16 KiB", "one workgroup per chunk"),
        ("4 KiB", "persistent grid (8 per CU)")) for nt in ("", ", nt"))       # mfx_store_ceiling shapes 0..7

    def store_ceiling(self, total_bytes, shape, group=0):
        """GB/s of a write-only float4 stream of total_bytes over this batch's view buffer of `group` (wrapping;
        mfx_store_ceiling, shape index into STORE_SHAPES) on the engine's stream.  Overwrites the views: call it
        only after their last use."""
        ptr, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._check(self._dll.mfx_battle_rollout_buffer(self.game, b"view", group, ctypes.byref(ptr), ctypes.byref(n)),
                    "rollout_buffer")
        ms = ctypes.c_float()
        self._dll.mfx_store_ceiling.restype = ctypes.c_int
        self._check(self._dll.mfx_store_ceiling(ptr, n, ctypes.c_size_t(int(total_bytes)), int(shape),
                                                ctypes.c_void_p(self.stream_handle()), ctypes.byref(ms)),
                    "store_ceiling")
        return (int(total_bytes) // 4096 * 4096) / (ms.value * 1e-3) / 1e9

    def view_support(self, group):
        """uint8 [view_h * view_w * n_ch] (the view's NHWC order): 1 where group `group`'s observation view can be
        non-zero, 0 where it is always zero (cells outside the view range carry only the minimap channels)."""
        n = int(np.prod(self.env.get_view_space(self.handles[group])))
        mask = np.zeros(n, dtype=np.uint8)
        self._dll.mfx_battle_view_support.restype = ctypes.c_int
        self._check(self._dll.mfx_battle_view_support(self.game, int(group), mask.ctypes.data_as(ctypes.c_void_p), n),
                    "view_support")
        return mask

    def rollout_copy(self, name, dst, group=0, nbytes=None):
        """Copy a device rollout buffer into dst (numpy array or torch tensor, host or device)."""
        ptr = dst.data_ptr() if hasattr(dst, "data_ptr") else dst.ctypes.data
        size = nbytes if nbytes is not None else (dst.numel() * dst.element_size() if hasattr(dst, "numel")
                                                  else dst.nbytes)
        self._check(self._dll.mfx_battle_rollout_copy(self.game, name.encode(), group, ctypes.c_void_p(ptr),
                                                      ctypes.c_size_t(size)), "rollout_copy")

    def rollout_copy_at(self, name, dst, offset, group=0, nbytes=None):
        """Copy bytes [offset, offset + nbytes) of a device rollout buffer into dst."""
        ptr = dst.data_ptr() if hasattr(dst, "data_ptr") else dst.ctypes.data
        size = nbytes if nbytes is not None else (dst.numel() * dst.element_size() if hasattr(dst, "numel")
                                                  else dst.nbytes)
        self._check(self._dll.mfx_battle_rollout_copy_at(self.game, name.encode(), group, ctypes.c_size_t(offset),
                                                         ctypes.c_void_p(ptr), ctypes.c_size_t(size)),
                    "rollout_copy_at")
