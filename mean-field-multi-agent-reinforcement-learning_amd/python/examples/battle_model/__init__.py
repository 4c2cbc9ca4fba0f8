"""Drop-in of the reference's examples/battle_model python side (algo, senario_battle) on
PyTorch-ROCm; the engine itself is the top-level `magent` drop-in."""
