"""Replay data path throughput: MemoryGroup.sample of the MF-Q learner
(examples/battle_model/algo/tools.py:239-262 -> mfrl_amd.algo.tools.MemoryGroup.sample): every column of a
minibatch gathered at random row indices (view, feature, action, reward, terminal, mask, mean action) and the
next-state columns at idx + 1 -- one mfx_rows_copy_shift launch (csrc/replay_kernels.hip; --two-launches: the
current and next-state columns as two launches, round 6's form).  Sampled rows per second
over a large batch, the kernel's bytes (read + write of every row) against the HBM roofline, next to the
reference's numpy fancy indexing (MetaBuffer.sample, tools.py:38-40) of the same columns on one host thread.

    python scripts/bench_replay.py [--capacity C] [--batch B]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))

ap = argparse.ArgumentParser()
ap.add_argument("--capacity", type=int, default=1 << 18)
ap.add_argument("--batch", type=int, default=1 << 16)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--cpu-seconds", type=float, default=10.0)
ap.add_argument("--two-launches", action="store_true")
a = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402
from mfrl_amd.replay import rows_copy  # noqa: E402

VIEW, FEAT, NA = 1183, 34, 21
C, B = a.capacity, a.batch
spec = [("obs", (VIEW,), torch.float32), ("feat", (FEAT,), torch.float32), ("act", (), torch.int32),
        ("rew", (), torch.float32), ("term", (), torch.bool), ("mask", (), torch.bool), ("prob", (NA,), torch.float32)]
g = torch.Generator(device="cuda").manual_seed(3)
bufs = {k: (torch.rand((C,) + s, device="cuda", generator=g) * 3).to(d) for k, s, d in spec}
cur = [k for k, _, _ in spec]
nxt = ["obs", "feat", "prob"]
outs_c = [torch.empty((B,) + tuple(bufs[k].shape[1:]), dtype=bufs[k].dtype, device="cuda") for k in cur]
outs_n = [torch.empty((B,) + tuple(bufs[k].shape[1:]), dtype=bufs[k].dtype, device="cuda") for k in nxt]
row_c = sum(bufs[k][0].numel() * bufs[k].element_size() for k in cur)
row_n = sum(bufs[k][0].numel() * bufs[k].element_size() for k in nxt)
bytes_per_row = 2 * (row_c + row_n)                  # every byte read once and written once
idx = torch.randint(0, C, (B,), device="cuda", generator=g)
nidx = (idx + 1) % C


def sample():
    if a.two_launches:
        rows_copy(outs_c, [bufs[k] for k in cur], idx, src_mod=C)
        rows_copy(outs_n, [bufs[k] for k in nxt], nidx, src_mod=C)
    else:
        rows_copy(outs_c + outs_n, [bufs[k] for k in cur + nxt], idx, src_mod=C,
                  shift_mask=((1 << len(nxt)) - 1) << len(cur), shift=1)


for _ in range(3):
    sample()
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
t0 = time.perf_counter()
for s, e in ev:
    s.record()
    sample()
    e.record()
torch.cuda.synchronize()
wall = time.perf_counter() - t0
ms = sorted(s.elapsed_time(e) for s, e in ev)
med = ms[len(ms) // 2]
# parity of one sample against torch indexing (the kernel must move the same bytes)
for o, k in zip(outs_c, cur):
    assert torch.equal(o, bufs[k][idx]), k
for o, k in zip(outs_n, nxt):
    assert torch.equal(o, bufs[k][nidx]), k
# CPU: the reference's numpy fancy indexing of the same columns (MetaBuffer.sample = self._data[idx])
Cc = min(C, 1 << 16)
host = {k: bufs[k][:Cc].cpu().numpy() for k in cur}
rs = np.random.RandomState(5)
t0, rows = time.perf_counter(), 0
while time.perf_counter() - t0 < a.cpu_seconds:
    hi = rs.choice(Cc, size=4096)
    hn = (hi + 1) % Cc
    _ = [host[k][hi] for k in cur]
    _ = [host[k][hn] for k in nxt]
    rows += len(hi)
cdt = time.perf_counter() - t0
line = {"metric": "replay minibatch rows sampled/sec (MemoryGroup.sample, MF-Q columns)", "value": B / (med * 1e-3),
        "unit": "rows/s", "batch": B, "capacity": C, "reps": a.reps, "ms_per_sample_median": med,
        "wall_rows_per_s": B * a.reps / wall,
        "roofline": {"bound": "hbm", "achieved": bytes_per_row * B / (med * 1e-3) / 1e9, "peak": 8000.0, "unit": "GB/s",
                     "frac": bytes_per_row * B / (med * 1e-3) / 1e9 / 8000.0, "bytes_per_unit": bytes_per_row,
                     "kernel": "k_rows_pipe x2 (current columns, next-state columns)" if a.two_launches else
                     "k_rows_pipe (current + next-state columns, one launch)"},
        "cpu_baseline": {"value": rows / cdt, "unit": "rows/s", "cores": 1, "kind": "port",
                         "sample": "numpy fancy indexing of the same 7 + 3 columns, 4096-row draws from a %d-row host "
                                   "buffer for %.0f s (MetaBuffer.sample's self._data[idx])" % (Cc, a.cpu_seconds)}}
print(json.dumps(line))
