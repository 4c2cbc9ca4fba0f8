"""The learned-policy forwards alone (k_acnet: ActorCritic / MFAC, algo/ac.py; k_qnet_conv + k_qnet_head: the
mean-field QNet, algo/base.py) on n random bench-shape agents (13x13x7 views, 34 features, 21 actions): HIP-event time
per forward, TFLOP/s over the policy path's FLOPs and the fraction of the f32 MFMA peak.  Random-init torch modules,
random inputs (the MFMA work does not depend on the values).

    python scripts/bench_policy.py [--net acnet|qnet] [--n 262144] [--reps 10] [--support]

--support (acnet): the Battle view's input support (mfx_battle_view_support's mask for 13x13x7: 903 inputs), the
random views zeroed outside it; FLOPs counted as executed (the view layer over 903 inputs), beside the dense count."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, REPO)

ap = argparse.ArgumentParser()
ap.add_argument("--net", choices=("acnet", "qnet"), default="acnet")
ap.add_argument("--n", type=int, default=262144)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--support", action="store_true")
a = ap.parse_args()

import torch  # noqa: E402
from bench import ACNET_FLOP_PER_AGENT, F32_MFMA_PEAK_TFS, QNET_FLOP_PER_AGENT  # noqa: E402
from mfrl_amd.algo.nets import ACNet, QNet  # noqa: E402
from mfrl_amd.policy import ACNetHIP, QNetHIP  # noqa: E402

torch.cuda.set_device(0)
torch.manual_seed(3)
n = a.n
view = torch.rand((n, 13, 13, 7), device="cuda")
feat = torch.rand((n, 34), device="cuda")
prob = torch.rand((n, 21), device="cuda")
flop_dense = None
if a.net == "acnet":
    hip = ACNetHIP((13, 13, 7), (34,), 21, True).load(ACNet((13, 13, 7), (34,), 21, use_mf=True).cuda())
    run = lambda k: hip.forward(view, feat, want_policy=False, seed=1, step=k)  # noqa: E731
    flop = flop_dense = ACNET_FLOP_PER_AGENT
    if a.support:
        import numpy as np
        y, x = np.mgrid[-6:7, -6:7]
        circle = (x * x + y * y <= 36)[:, :, None]
        mask = (circle | (np.arange(7) % 3 == 0)[None, None, :] & (np.arange(7) > 0)[None, None, :]).reshape(-1)
        assert int(mask.sum()) == 903
        view *= torch.from_numpy(mask.astype(np.float32).reshape(13, 13, 7)).cuda()
        hip.set_input_support(mask.astype(np.uint8))
        flop = 2 * (903 * 256 + 34 * 256 + 512 * 512 + 512 * 21)
else:
    hip = QNetHIP((13, 13, 7), (34,), 21, True).load(QNet((13, 13, 7), (34,), 21, True).cuda())
    run = lambda k: hip.forward(view, feat, prob)  # noqa: E731
    flop = QNET_FLOP_PER_AGENT
for k in range(2):
    run(k)
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
for k in range(a.reps):
    ev[k][0].record()
    run(k)
    ev[k][1].record()
torch.cuda.synchronize()
ms = sorted(x.elapsed_time(y) for x, y in ev)
med = ms[len(ms) // 2]
tfs = flop * n / (med * 1e-3) / 1e12
print(json.dumps({"net": a.net, "n": n, "ms_median": med, "ms_min": ms[0], "tflops": tfs, "frac": tfs / F32_MFMA_PEAK_TFS,
                  "flop_per_agent": flop, "flop_per_agent_dense": flop_dense, "support": a.support,
                  "env": {k: v for k, v in os.environ.items() if k.startswith("MFX_")}}),
      flush=True)
