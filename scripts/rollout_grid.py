"""Print the fused rollout's persistent grid and LDS bytes for the bench config (MAGENT_LIB picks the build)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import battle_driver as bd  # noqa: E402
from mfrl_amd.battle import BattleBatch  # noqa: E402

eng = BattleBatch(64, 16384, stream=torch.cuda.current_stream())
left, right = bd.block_positions(64, 128)
eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=1)
print(os.environ.get("MAGENT_LIB", "default"), "grid, lds =", eng.rollout_info(),
      "CUs", torch.cuda.get_device_properties(0).multi_processor_count)
