"""PyTorch-ROCm drop-in of the reference's examples/battle_model/algo (TF1): same classes, same
spawn_ai factory and call signatures (`sess` is accepted and ignored).  SURVEY.md 8(f) rows 1-2:
policy forward and replay on the device; the MF-Q target and the MF-AC returns run in this
library's HIP kernels."""
from . import ac
from . import q_learning
from . import tools

AC = ac.ActorCritic
MFAC = ac.MFAC
IL = q_learning.DQN
MFQ = q_learning.MFQ


def spawn_ai(algo_name, sess, env, handle, human_name, max_steps, memory_size=80000):
    """algo/__init__.py:10-19 (memory_size: the replay rows of MFQ / IL; 80000 there)."""
    if algo_name == "mfq":
        model = MFQ(sess, human_name, handle, env, max_steps, memory_size=memory_size)
    elif algo_name == "mfac":
        model = MFAC(sess, human_name, handle, env)
    elif algo_name == "ac":
        model = AC(sess, human_name, handle, env)
    elif algo_name == "il":
        model = IL(sess, human_name, handle, env, max_steps, memory_size=memory_size)
    else:
        raise ValueError("unknown algo %r" % algo_name)
    return model
