"""The C-ABI library on a machine without a GPU: it loads, exports every symbol that
include/magent_amd.h declares, and fails loudly (EngineError) instead of computing anything."""
import ctypes
import os
import re
import subprocess

import pytest

import common

HEADER = os.path.join(common.REPO, "include", "magent_amd.h")


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(common.HIP_LIB):
        subprocess.run(["make", "-s", "-C", common.PKG], check=True)
    return common.HIP_LIB


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(?:int|const char \*)\s*\**\s*(\w+)\s*\(", text)))


def test_header_declares_reference_abi():
    names = declared()
    ref = ["env_new_game", "env_delete_game", "env_config_game", "env_reset", "env_get_observation",
           "env_set_action", "env_step", "env_get_reward", "env_get_info", "env_render", "env_render_next_file",
           "gridworld_register_agent_type", "gridworld_new_group", "gridworld_add_agents", "gridworld_clear_dead",
           "gridworld_set_goal", "gridworld_define_agent_symbol", "gridworld_define_event_node",
           "gridworld_add_reward_rule"]
    assert set(ref) <= set(names)


def test_library_exports_every_declared_symbol(built):
    out = subprocess.run(["nm", "-D", "--defined-only", built], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing


def test_library_loads_and_reports_without_gpu(built):
    dll = ctypes.CDLL(built, mode=ctypes.RTLD_LOCAL)
    dll.mfx_build_info.restype = ctypes.c_char_p
    assert b"gfx950" in dll.mfx_build_info()
    assert dll.mfx_device_count() >= 0


def test_engine_fails_loudly_without_gpu(built):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import magent
    env = magent.GridWorld("battle", map_size=20, lib=magent.load_library(built))
    with pytest.raises(magent.EngineError):
        env.reset()


def test_dropin_rejects_unsupported_config(built):
    """The reward event 'align' is the one DSL form the engine refuses (the reference reads uninitialised
    counters for it); the rules are compiled at reset, before any device work, so
    the refusal shows without a GPU.  can_absorb types are accepted (tests/test_absorb.py)."""
    import magent
    gw = magent.gridworld
    cfg = gw.Config()
    cfg.set({"map_width": 10, "map_height": 10})
    t = cfg.register_agent_type("blob", {"width": 1, "length": 1, "hp": 1, "speed": 1, "can_absorb": True,
                                         "view_range": gw.CircleRange(1), "attack_range": gw.CircleRange(1)})
    g = cfg.add_group(t)
    cfg.add_reward_rule(gw.Event(gw.AgentSymbol(g, "all"), "align"), receiver=gw.AgentSymbol(g, "all"), value=1.0)
    env = magent.GridWorld(cfg, lib=magent.load_library(built))
    with pytest.raises(magent.EngineError, match="align"):
        env.reset()


def test_battle_view_support_without_gpu(built):
    """mfx_battle_view_support: the Battle view (13 x 13 x 7) can be non-zero in every channel of the 113 cells of
    the radius-6 view circle and in the two minimap channels (3, 6) of every cell; nothing else is ever written
    (Map.cc:130-218, GridWorld.cc:396-409).  No device work: the parameters compile on the host."""
    import numpy as np
    import magent
    env = magent.GridWorld("battle", map_size=64, lib=magent.load_library(built))
    h = env.get_handles()
    dll = env._lib.dll
    dll.mfx_battle_view_support.restype = ctypes.c_int
    for g in range(2):
        m = np.zeros(13 * 13 * 7, dtype=np.uint8)
        assert dll.mfx_battle_view_support(env.game, g, m.ctypes.data_as(ctypes.c_void_p), m.size) == 0
        m = m.reshape(13, 13, 7)
        y, x = np.mgrid[-6:7, -6:7]
        circle = (x * x + y * y <= 36).astype(np.uint8)
        assert circle.sum() == 113
        for ch in range(7):
            assert np.array_equal(m[:, :, ch], np.ones_like(circle) if ch in (3, 6) else circle), ch
        assert int(m.sum()) == 903
    bad = np.zeros(10, dtype=np.uint8)
    assert dll.mfx_battle_view_support(env.game, 0, bad.ctypes.data_as(ctypes.c_void_p), bad.size) != 0
