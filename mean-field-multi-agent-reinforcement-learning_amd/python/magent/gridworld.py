"""GridWorld: python surface of the Battle engine (reference python/magent/gridworld.py).

Same classes and methods as the reference wrapper -- GridWorld, Config, EventNode/Event,
AgentSymbol, CircleRange, SectorRange -- issuing the same C-ABI calls, so scripts written
against the reference (senario_battle.play, train_battle.py) run unchanged.  Differences:
engine calls are checked (an engine error raises magent.EngineError instead of aborting
the process) and ``GridWorld(..., lib=...)`` may select another build of the ABI.
"""
import ctypes
import importlib
import os

import numpy as np

from .c_lib import EngineError, get_lib, as_float_c_array, as_int32_c_array
from .environment import Environment

_CONFIG_TYPES = {
    "map_width": int, "map_height": int, "embedding_size": int,
    "food_mode": bool, "turn_mode": bool, "minimap_mode": bool, "revive_mode": bool, "goal_mode": bool,
    "render_dir": str,
}


class _Engine:
    """Owner of one engine handle: env_delete_game runs when the GridWorld and every observation view
    handed out by get_observation (which point into the engine's pinned memory) are gone."""
    __slots__ = ("lib", "game")

    def __init__(self, lib, game):
        self.lib, self.game = lib, game

    def __del__(self):
        if self.game is not None and self.game.value:
            self.lib.dll.env_delete_game(self.game)
            self.game = None


class GridWorld(Environment):
    OBS_INDEX_VIEW = 0
    OBS_INDEX_HP = 1

    def __init__(self, config, lib=None, **kwargs):
        """config: a Config, or the name of a builtin config (magent/builtin/config/<name>.py)
        whose get_config(**kwargs) builds one (gridworld.py:22-177 of the reference)."""
        Environment.__init__(self)
        if isinstance(config, str):
            try:
                mod = importlib.import_module("magent.builtin.config." + config)
            except ImportError:
                raise BaseException('unknown built-in game "%s"' % config)
            config = mod.get_config(**kwargs)
        self._lib = lib if lib is not None else get_lib()
        L = self._lib

        game = ctypes.c_void_p()
        L.env_new_game(ctypes.byref(game), b"GridWorld")
        self.game = game
        self._engine = _Engine(L, game)      # deletes the engine once neither this env nor a view needs it

        for key, value in config.config_dict.items():
            kind = _CONFIG_TYPES[key]
            if kind is int:
                L.env_config_game(self.game, key.encode("ascii"), ctypes.byref(ctypes.c_int(value)))
            elif kind is bool:
                L.env_config_game(self.game, key.encode("ascii"), ctypes.byref(ctypes.c_bool(value)))
            else:
                L.env_config_game(self.game, key.encode("ascii"), ctypes.c_char_p(str(value).encode("ascii")))

        for name, attrs in config.agent_type_dict.items():
            args = {}
            for key, val in attrs.items():
                if key in ("view_range", "attack_range"):
                    prefix = key.split("_")[0]
                    args[prefix + "_radius"] = val.radius
                    args[prefix + "_angle"] = val.angle
                else:
                    args[key] = val
            n = len(args)
            keys = (ctypes.c_char_p * n)(*[k.encode("ascii") for k in args])
            values = (ctypes.c_float * n)(*[float(v) for v in args.values()])
            L.gridworld_register_agent_type(self.game, name.encode("ascii"), n, keys, values)

        self._serialize_event_exp(config)

        self.group_handles = []
        for type_name in config.groups:
            handle = ctypes.c_int32()
            L.gridworld_new_group(self.game, type_name.encode("ascii"), ctypes.byref(handle))
            self.group_handles.append(handle)

        self._init_obs_buf()
        # engines that hold the drop-in step's observation in pinned memory hand it out without a copy
        self._obs_view = getattr(L.dll, "mfx_env_observation_view", None) if hasattr(L, "dll") else None
        if self._obs_view is not None:
            vp = ctypes.POINTER(ctypes.c_void_p)
            ip = ctypes.POINTER(ctypes.c_int32)
            self._obs_view.argtypes = [ctypes.c_void_p, ctypes.c_int, vp, vp, ip, ip]
            self._obs_view.restype = ctypes.c_int
            self._ov_out = (ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int32(), ctypes.c_int32())
            self._ov_ref = tuple(ctypes.byref(x) for x in self._ov_out)
            self._ov_blocks = {}                 # (address, rows, shape) -> array over that pinned block
        # engines holding env 0's record on the host answer each getter in one call (mfx_env_get_rows) where
        # the reference's wrapper makes two (env_get_info("num"), then the field)
        self._rows = getattr(L.dll, "mfx_env_get_rows", None) if hasattr(L, "dll") else None
        if self._rows is not None:
            self._rows.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
            self._rows.restype = ctypes.c_int
            self._rows_cap = 256
        self.view_space, self.feature_space, self.action_space = {}, {}, {}
        buf = np.empty((3,), dtype=np.int32)
        for h in self.group_handles:
            L.env_get_info(self.game, h.value, b"view_space", buf.ctypes.data_as(ctypes.c_void_p))
            self.view_space[h.value] = (int(buf[0]), int(buf[1]), int(buf[2]))
            L.env_get_info(self.game, h.value, b"feature_space", buf.ctypes.data_as(ctypes.c_void_p))
            self.feature_space[h.value] = (int(buf[0]),)
            L.env_get_info(self.game, h.value, b"action_space", buf.ctypes.data_as(ctypes.c_void_p))
            self.action_space[h.value] = (int(buf[0]),)

    # ------------------------------------------------------------------ lifecycle
    def reset(self):
        self._lib.env_reset(self.game)

    def add_walls(self, method, **kwargs):
        kwargs["dir"] = 0
        self.add_agents(-1, method, **kwargs)

    def new_group(self, name):
        handle = ctypes.c_int32()
        self._lib.gridworld_new_group(self.game, name.encode("ascii"), ctypes.byref(handle))
        return handle

    def add_agents(self, handle, method, **kwargs):
        g = _hv(handle)
        L = self._lib
        null = ctypes.POINTER(ctypes.c_int32)()
        if method == "random":
            L.gridworld_add_agents(self.game, g, int(kwargs["n"]), b"random", null, null, null)
        elif method == "custom":
            pos = np.array(kwargs["pos"], dtype=np.int32)
            if len(pos) <= 0:
                return
            xs = np.ascontiguousarray(pos[:, 0])
            ys = np.ascontiguousarray(pos[:, 1])
            dirs = np.ascontiguousarray(pos[:, 2]) if pos.shape[1] == 3 else np.zeros(len(pos), np.int32)
            L.gridworld_add_agents(self.game, g, len(pos), b"custom", as_int32_c_array(xs),
                                   as_int32_c_array(ys), as_int32_c_array(dirs))
        elif method == "fill":
            x, y = kwargs["pos"][0], kwargs["pos"][1]
            width, height = kwargs["size"][0], kwargs["size"][1]
            direction = kwargs.get("dir", np.zeros_like(x))
            bind = np.array([x, y, width, height, direction], dtype=np.int32)
            L.gridworld_add_agents(self.game, g, 0, b"fill", as_int32_c_array(bind), null, null)
        else:
            raise ValueError("unknown placement method %r" % method)

    # ------------------------------------------------------------------ run
    def _init_obs_buf(self):
        self.obs_bufs = [{}, {}]

    def _get_obs_buf(self, group, key, shape, dtype):
        """The same array is returned on every call and resized in place (reference :282-295)."""
        bufs = self.obs_bufs[key]
        if group in bufs:
            ret = bufs[group]
            if ret.shape != shape:
                ret.resize(shape, refcheck=False)
        else:
            ret = bufs[group] = np.empty(shape=shape, dtype=dtype)
        return ret

    def _block(self, addr, rows, space):
        """float32 [rows, *space] array over the engine-owned pinned block at addr (made once per block);
        it keeps the engine (self._engine), not this env, alive."""
        key = (addr, rows, space)
        b = self._ov_blocks.get(key)
        if b is None:
            count = rows
            for d in space:
                count *= d
            buf = (ctypes.c_float * count).from_address(addr)
            buf._owner = self._engine
            b = self._ov_blocks[key] = np.frombuffer(buf, dtype=np.float32).reshape((rows,) + space)
        return b

    def get_observation(self, handle):
        """(views [n, H, W, C] float32, features [n, F] float32) of every agent of the group.

        After a drop-in step the engine already holds them in pinned memory and the arrays are views
        of it (no copy); like the reference's reused buffers they are overwritten later -- here by the
        step after next, which leaves them valid through the replay push that follows env.step()."""
        g = _hv(handle)
        if self._obs_view is not None:
            ref = self._ov_ref
            r = self._obs_view(self.game, g, ref[0], ref[1], ref[2], ref[3])
            if r == 0:
                vp, fp, n, rows = self._ov_out
                n, rows = n.value, rows.value
                return (self._block(vp.value, rows, self.view_space[g])[:n],
                        self._block(fp.value, rows, self.feature_space[g])[:n])
            if r < 0:
                raise EngineError("mfx_env_observation_view failed (%d): %s"
                                  % (r, self._lib.dll.mfx_last_error().decode()))
        n = self.get_num(handle)
        view = self._get_obs_buf(g, self.OBS_INDEX_VIEW, (n,) + self.view_space[g], np.float32)
        feat = self._get_obs_buf(g, self.OBS_INDEX_HP, (n,) + self.feature_space[g], np.float32)
        bufs = (ctypes.POINTER(ctypes.c_float) * 2)()
        bufs[0] = as_float_c_array(view)
        bufs[1] = as_float_c_array(feat)
        self._lib.env_get_observation(self.game, g, bufs)
        return view, feat

    def set_action(self, handle, actions):
        assert isinstance(actions, np.ndarray)
        assert actions.dtype == np.int32
        actions = np.ascontiguousarray(actions)
        self._lib.env_set_action(self.game, _hv(handle), actions.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))

    def step(self):
        done = ctypes.c_int32()
        self._lib.env_step(self.game, ctypes.byref(done))
        return bool(done.value)

    def get_reward(self, handle):
        if self._rows is not None:
            return self._get_rows(handle, 1, np.float32)
        buf = np.empty((self.get_num(handle),), dtype=np.float32)
        self._lib.env_get_reward(self.game, _hv(handle), as_float_c_array(buf))
        return buf

    def clear_dead(self):
        self._lib.gridworld_clear_dead(self.game)

    # ------------------------------------------------------------------ info
    def get_handles(self):
        return self.group_handles

    def _get_rows(self, handle, what, dtype, tail=()):
        """A fresh array of the group's rows of field `what` (mfx_env_get_rows: 0 id, 1 reward, 2 alive, 3 pos)."""
        g = _hv(handle)
        while True:
            buf = np.empty((self._rows_cap,) + tail, dtype=dtype)
            n = self._rows(self.game, g, what, buf.__array_interface__["data"][0], self._rows_cap)
            if n < 0:
                raise EngineError("mfx_env_get_rows failed: %s" % self._lib.dll.mfx_last_error().decode())
            if n <= self._rows_cap:
                return buf[:n]
            self._rows_cap = max(n, 2 * self._rows_cap)

    def get_num(self, handle):
        if self._rows is not None:
            n = self._rows(self.game, _hv(handle), -1, None, 0)
            if n < 0:
                raise EngineError("mfx_env_get_rows failed: %s" % self._lib.dll.mfx_last_error().decode())
            return n
        num = ctypes.c_int32()
        self._lib.env_get_info(self.game, _hv(handle), b"num", ctypes.byref(num))
        return num.value

    def get_action_space(self, handle):
        return self.action_space[_hv(handle)]

    def get_view_space(self, handle):
        return self.view_space[_hv(handle)]

    def get_feature_space(self, handle):
        return self.feature_space[_hv(handle)]

    def _info_array(self, handle, name, shape, dtype):
        buf = np.empty(shape, dtype=dtype)
        self._lib.env_get_info(self.game, _hv(handle), name, buf.ctypes.data_as(ctypes.c_void_p))
        return buf

    def get_agent_id(self, handle):
        if self._rows is not None:
            return self._get_rows(handle, 0, np.int32)
        return self._info_array(handle, b"id", (self.get_num(handle),), np.int32)

    def get_alive(self, handle):
        if self._rows is not None:
            return self._get_rows(handle, 2, np.bool_)
        return self._info_array(handle, b"alive", (self.get_num(handle),), np.bool_)

    def get_pos(self, handle):
        if self._rows is not None:
            return self._get_rows(handle, 3, np.int32, (2,))
        return self._info_array(handle, b"pos", (self.get_num(handle), 2), np.int32)

    def get_view2attack(self, handle):
        """(attack_base, int32[view_h, view_w] with the attack index of each attackable cell, else -1)."""
        buf = self._info_array(handle, b"view2attack", self.get_view_space(handle)[0:2], np.int32)
        base = ctypes.c_int32()
        self._lib.env_get_info(self.game, _hv(handle), b"attack_base", ctypes.byref(base))
        return base.value, buf

    def set_seed(self, seed):
        self._lib.env_config_game(self.game, b"seed", ctypes.byref(ctypes.c_int(seed)))

    # ------------------------------------------------------------------ get_info extras (gridworld.py:486-636)
    def _call_info(self, group, name, buf):
        self._lib.env_get_info(self.game, group, name, buf.ctypes.data_as(ctypes.c_void_p))   # checked
        return buf

    def get_mean_info(self, handle):
        """float32 [2 + n_action]: mean x, mean y, action frequencies (deprecated in the reference)."""
        buf = np.empty(2 + self.get_action_space(handle)[0], dtype=np.float32)
        return self._call_info(_hv(handle), b"mean_info", buf)

    def get_global_minimap(self, height, width):
        """float32 [height, width, n_group]: per-group agent density over a downsampled map."""
        buf = np.empty((height, width, len(self.group_handles)), dtype=np.float32)
        buf[0, 0, 0] = height
        buf[0, 0, 1] = width
        return self._call_info(-1, b"global_minimap", buf)

    def _get_groups_info(self):
        buf = np.empty((len(self.group_handles), 5), dtype=np.int32)
        return self._call_info(-1, b"groups_info", buf)

    def _get_walls_info(self):
        buf = np.empty((100 * 100, 2), dtype=np.int32)
        self._call_info(-1, b"walls_info", buf)
        return buf[1:1 + buf[0, 0]]

    def _get_render_info(self, x_range, y_range):
        n = sum(self.get_num(h) for h in self.group_handles)
        buf = np.empty((n + 1, 4), dtype=np.int32)
        buf[0] = x_range[0], y_range[0], x_range[1], y_range[1]
        self._call_info(-1, b"render_window_info", buf)
        agent_ct, attack_event_ct = buf[0, 0], buf[0, 1]
        agent_info = {int(item[0]): [int(item[1]), int(item[2]), int(item[3])] for item in buf[1:1 + agent_ct]}
        events = np.empty((attack_event_ct, 3), dtype=np.int32)
        self._call_info(-1, b"attack_event", events)
        return agent_info, events

    # ------------------------------------------------------------------ render (out of scope: no-op)
    def set_render_dir(self, name):
        if not os.path.exists(name):
            os.makedirs(name, exist_ok=True)
        self._lib.env_config_game(self.game, b"render_dir", ctypes.c_char_p(name.encode("ascii")))

    def render(self):
        self._lib.env_render(self.game)

    def __del__(self):
        self._engine = None                  # the engine goes when the last observation view does

    # ------------------------------------------------------------------ reward description
    def _serialize_event_exp(self, config):
        """Number the symbols and event nodes and send them to the engine (reference :636-722)."""
        symbol_no, node_no = {}, {}

        def number_symbol(sym):
            if sym not in symbol_no:
                symbol_no[sym] = len(symbol_no)

        def walk_symbols(node):
            for item in node.inputs:
                if isinstance(item, EventNode):
                    walk_symbols(item)
                elif isinstance(item, AgentSymbol):
                    number_symbol(item)

        def walk_nodes(node):
            if node not in node_no:
                node_no[node] = len(node_no)
            for item in node.inputs:
                if isinstance(item, EventNode):
                    walk_nodes(item)

        for on, receivers, _values, _terminal in config.reward_rules:
            for sym in receivers:
                number_symbol(sym)
            walk_symbols(on)
        for rule in config.reward_rules:
            walk_nodes(rule[0])

        L = self._lib
        for sym, no in symbol_no.items():
            L.gridworld_define_agent_symbol(self.game, no, sym.group, sym.index)
        for node, no in node_no.items():
            inputs = np.array([node_no[x] if isinstance(x, EventNode) else
                               symbol_no[x] if isinstance(x, AgentSymbol) else int(x)
                               for x in node.inputs], dtype=np.int32)
            L.gridworld_define_event_node(self.game, no, node.op, as_int32_c_array(inputs), len(inputs))
        for on, receivers, values, terminal in config.reward_rules:
            recv = np.array([symbol_no[x] for x in receivers], dtype=np.int32)
            if len(values) == 1 and values[0] == "auto":
                vals = np.zeros(len(recv), dtype=np.float32)
            else:
                vals = np.array(values, dtype=np.float32)
            L.gridworld_add_reward_rule(self.game, node_no[on], as_int32_c_array(recv), as_float_c_array(vals),
                                        len(recv), bool(terminal), False)


def _hv(handle):
    return handle.value if isinstance(handle, ctypes.c_int32) else int(handle)


# ====================================================================== reward DSL
class EventNode:
    """AST node of a reward-trigger expression (reference gridworld.py:731-830)."""
    OP_AND, OP_OR, OP_NOT = 0, 1, 2
    OP_KILL, OP_AT, OP_IN, OP_COLLIDE, OP_ATTACK, OP_DIE, OP_IN_A_LINE, OP_ALIGN = 3, 4, 5, 6, 7, 8, 9, 10

    _BINARY = {"kill": OP_KILL, "attack": OP_ATTACK, "collide": OP_COLLIDE}
    _UNARY = {"die": OP_DIE, "in_a_line": OP_IN_A_LINE, "align": OP_ALIGN}

    def __init__(self):
        self.op = None
        self.predicate = None
        self.inputs = []

    def __call__(self, subject, predicate, *args):
        node = EventNode()
        node.predicate = predicate
        if predicate in self._BINARY:
            node.op, node.inputs = self._BINARY[predicate], [subject, args[0]]
        elif predicate in self._UNARY:
            node.op, node.inputs = self._UNARY[predicate], [subject]
        elif predicate == "at":
            node.op, node.inputs = EventNode.OP_AT, [subject, args[0][0], args[0][1]]
        elif predicate == "in":
            (ax, ay), (bx, by) = args[0][0], args[0][1]
            node.op = EventNode.OP_IN
            node.inputs = [subject, min(ax, bx), min(ay, by), max(ax, bx), max(ay, by)]
        else:
            raise Exception("invalid predicate of event " + predicate)
        return node

    def _combine(self, op, *others):
        node = EventNode()
        node.op, node.inputs = op, [self, *others]
        return node

    def __and__(self, other):
        return self._combine(EventNode.OP_AND, other)

    def __or__(self, other):
        return self._combine(EventNode.OP_OR, other)

    def __invert__(self):
        return self._combine(EventNode.OP_NOT)


Event = EventNode()


class AgentSymbol:
    """Some agents of a group: index 'any' (-1), 'all' (-2) or a fixed index."""

    def __init__(self, group, index):
        self.group = group if group is not None else -1
        if index == "any":
            self.index = -1
        elif index == "all":
            self.index = -2
        else:
            assert isinstance(index, int), "index must be a deterministic int"
            self.index = index

    def __str__(self):
        return "agent(%d,%d)" % (self.group, self.index)


class Config:
    """Game configuration: global keys, agent types, groups, reward rules (reference :867-977)."""

    def __init__(self):
        self.config_dict = {}
        self.agent_type_dict = {}
        self.groups = []
        self.reward_rules = []

    def set(self, args):
        self.config_dict.update(args)

    def register_agent_type(self, name, attr):
        if name in self.agent_type_dict:
            raise Exception("type name %s already exists" % name)
        self.agent_type_dict[name] = attr
        return name

    def add_group(self, agent_type):
        self.groups.append(agent_type)
        return len(self.groups) - 1

    def add_reward_rule(self, on, receiver, value, terminal=False):
        if not isinstance(receiver, (tuple, list)):
            assert not isinstance(value, (tuple, list))
            receiver, value = [receiver], [value]
        if len(receiver) != len(value):
            raise Exception("the length of receiver and value should be equal")
        self.reward_rules.append([on, list(receiver), list(value), terminal])


class CircleRange:
    def __init__(self, radius):
        self.radius = radius
        self.angle = 360

    def __str__(self):
        return "circle(%g)" % self.radius


class SectorRange:
    def __init__(self, radius, angle):
        self.radius = radius
        self.angle = angle
        if self.angle >= 180:
            raise Exception("the angle of a sector should be smaller than 180 degree")

    def __str__(self):
        return "sector(%g, %g)" % (self.radius, self.angle)
