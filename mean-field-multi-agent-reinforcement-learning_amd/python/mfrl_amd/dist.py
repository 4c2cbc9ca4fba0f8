"""Multi-GPU plumbing of the throughput path: one process per GPU, envs sharded by rank.

Envs are independent, so the data path has no collective: each rank steps its
own E envs.  The only exchange is the episode statistics (a few floats per step) and the
bench's timing: max of the per-rank wall time, sum of the per-rank agent-steps.  Ising replicas shard the
same way (replica_block): each rank runs a contiguous block of replicas, replica r always with seed
seed0 + r, and one all-reduce of (sum of final order parameters, sum of steps, replicas) per run
(reduce_ising; main_MFQ_Ising.py:138-156 tracks the order parameter per episode)."""
import torch
import torch.distributed as dist


def env_seed(base, rank):
    """Every rank runs a different synthetic stream."""
    return base + 7919 * rank


def reduce_stats(stats):
    """Sum episode statistics [..., 4] (episodes, return g0, return g1, kills) over envs and ranks."""
    red = stats.reshape(-1, stats.shape[-1]).sum(0)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(red)
    return red


def reduce_timing(elapsed_s, units, device):
    """(max wall time over ranks, total units over ranks)."""
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    u = torch.tensor([float(units)], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
    return float(t.item()), float(u.item())


def replica_block(R, world, rank):
    """(first replica, count) of this rank's block of R replicas (the remainder to the low ranks)."""
    base, extra = divmod(R, world)
    count = base + (1 if rank < extra else 0)
    return rank * base + min(rank, extra), count


def reduce_ising(final_order, steps, device="cpu"):
    """[sum of the replicas' final order parameters, sum of their episode lengths, replicas] over every rank (one
    all-reduce); final_order / steps: this rank's per-replica values."""
    import numpy as np
    v = torch.tensor([float(np.sum(np.asarray(final_order, dtype=np.float64))), float(np.sum(steps)),
                      float(len(steps))], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(v)
    return v.tolist()
