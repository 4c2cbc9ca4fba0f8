"""The N>1 bench plumbing on CPU: world_size 2 over gloo (the GPU box uses RCCL through the same
calls).  Checks the max-over-ranks time, the summed agent-steps and the stats all-reduce."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mfrl_amd.dist import reduce_stats, reduce_timing, env_seed
    t, u = reduce_timing(1.0 + rank, 100 * (rank + 1), "cpu")
    stats = torch.full((3, 4), float(rank + 1), dtype=torch.float64)
    red = reduce_stats(stats)
    out[rank] = (t, u, red.tolist(), env_seed(1234, rank))
    dist.destroy_process_group()


def test_two_rank_reductions():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        t, u, red, seed = out[r]
        assert t == 2.0                 # max over ranks
        assert u == 300.0               # 100 + 200
        assert red == [9.0] * 4         # 3 envs x (1 + 2)
    assert out[0][3] != out[1][3]       # distinct per-rank streams
