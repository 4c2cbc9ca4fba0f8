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
