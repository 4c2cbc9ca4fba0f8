"""Drop-in replacement of the reference ``magent`` package (examples/battle_model/python/magent)
backed by the MI355X-native Battle engine (../../build/libmagent.so).

``import magent; env = magent.GridWorld('battle', map_size=40)`` works as in the reference;
scripts such as train_battle.py / senario_battle.play use the same calls.
"""
from . import gridworld
from .gridworld import GridWorld
from .c_lib import load_library, get_lib, EngineError

__all__ = ["GridWorld", "gridworld", "load_library", "get_lib", "EngineError"]
