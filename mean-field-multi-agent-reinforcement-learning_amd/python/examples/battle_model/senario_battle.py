"""`from examples.battle_model.senario_battle import play` -> mfrl_amd.algo.play."""
from mfrl_amd.algo.play import battle, generate_map, play, play_batched  # noqa: F401
