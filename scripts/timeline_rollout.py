"""Diagnostic: where a k_rollout launch's time goes at a given batch size (MFX_STAMPS build).

    MAGENT_LIB=.../build/libmagent_stamps.so python scripts/timeline_rollout.py --envs 8192 --substeps 20

For one launch of S steps after an episode cap of preparation: per env the install and write-back times
(s_memrealtime, 100 MHz), its workgroup and its agents at install.  Prints the envs in flight over the
launch, when the queue ran dry (the last install), the tail after it, the per-class unit durations, and
the per-workgroup busy time (sum of its units) against the launch span."""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import battle_driver as bd  # noqa: E402
from mfrl_amd.battle import BattleBatch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=8192)
ap.add_argument("--substeps", type=int, default=20)
ap.add_argument("--launches", type=int, default=2)
a = ap.parse_args()
E, S = a.envs, a.substeps
eng = BattleBatch(64, E, stream=torch.cuda.current_stream())
left, right = bd.block_positions(64, 128)
eng.rollout_init([left, right], max_steps=400, eps=0.2, seed=1234)
eng.rollout_substeps(S)
grid, lds = eng.rollout_info()
buf = torch.zeros(E * 32, dtype=torch.int64, device="cuda")
assert eng._dll.mfx_battle_set_stamp_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
eng.rollout_step(400 + 10)
torch.cuda.synchronize()
print("E %d, %d steps per launch, grid %d workgroups, LDS %d B" % (E, S, grid, lds))
for L in range(a.launches):
    buf.zero_()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    eng.rollout_step(S)
    ev[1].record()
    torch.cuda.synchronize()
    st = buf.view(E, 32).cpu().numpy().astype(np.int64)
    t0, t1, wg, n0 = st[:, 11], st[:, 12], st[:, 27], st[:, 29]
    base = t0.min()
    t0, t1 = (t0 - base) / 100.0, (t1 - base) / 100.0          # us
    span = t1.max()
    dur = t1 - t0
    print("launch %d: HIP events %.3f ms, stamped span %.3f ms; last install at %.3f ms (%.1f%%), tail %.3f ms"
          % (L, ev[0].elapsed_time(ev[1]), span / 1e3, t0.max() / 1e3, 100 * t0.max() / span, (span - t0.max()) / 1e3))
    bins = np.linspace(0, span, 21)
    inflight = [int(((t0 <= x) & (t1 > x)).sum()) for x in (bins[:-1] + bins[1:]) / 2]
    print("  envs in flight per 5%% of the span: %s" % inflight)
    for lo, hi in ((192, 10 ** 9), (128, 191), (64, 127), (33, 63), (0, 32)):
        sel = (n0 >= lo) & (n0 <= hi)
        if sel.any():
            print("  agents %4d-%-4s: %5d units, duration mean %7.1f us, max %7.1f us, started by %6.3f ms"
                  % (lo, hi if hi < 10 ** 9 else "", sel.sum(), dur[sel].mean(), dur[sel].max(), t0[sel].max() / 1e3))
    n_last = st[:, 16]                                          # agents at the launch's last step of the env
    light = n0 <= 63
    rst = light & (n_last > 128)                                # restarted inside the launch (256 placed again)
    print("  light units (<= 63 agents at install) that restarted inside the launch: %d of %d, duration mean %.1f us, "
          "max %.1f us; light units without a restart: mean %.1f us, max %.1f us"
          % (rst.sum(), light.sum(), dur[rst].mean() if rst.any() else 0.0, dur[rst].max() if rst.any() else 0.0,
             dur[light & ~rst].mean(), dur[light & ~rst].max()))
    slow = light & ~rst & (dur > 2000)
    if slow.any():
        print("  slow light units without a restart: %d, agents at install %s, finished at %s ms, workgroups %s"
              % (slow.sum(), n0[slow][:12].tolist(), np.round(t1[slow][:12] / 1e3, 2).tolist(), wg[slow][:12].tolist()))
    busy = np.bincount(wg, weights=dur, minlength=grid)
    last = np.zeros(grid)
    np.maximum.at(last, wg, t1)
    print("  per-workgroup busy / span: mean %.3f, min %.3f; workgroup finish time: min %.3f, median %.3f, max %.3f ms"
          % (busy.mean() / span, busy.min() / span, last.min() / 1e3, np.median(last) / 1e3, last.max() / 1e3))
    units = np.bincount(wg, minlength=grid)
    print("  units per workgroup: mean %.2f, min %d, max %d" % (units.mean(), units.min(), units.max()))
