"""Measured HBM ceilings on this box (torch's own kernels): write-only fill, copy, read-only sum.
Prints one JSON line; used to put k_rollout's achieved bandwidth next to what the card sustains."""
import json
import torch

n = 1 << 30                      # 4 GiB of fp32
x = torch.empty(n, device="cuda")
y = torch.empty(n, device="cuda")
x.fill_(1.0)
torch.cuda.synchronize()


def timed(fn, bytes_moved, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return bytes_moved * reps / (a.elapsed_time(b) * 1e-3) / 1e9


out = {"fill_GBps": timed(lambda: y.fill_(2.0), 4 * n),
       "copy_GBps": timed(lambda: y.copy_(x), 8 * n),
       "sum_GBps": timed(lambda: x.sum(), 4 * n)}
print(json.dumps(out))
