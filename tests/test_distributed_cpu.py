"""The N>1 bench plumbing on CPU: world_size 2 over gloo (the GPU box uses RCCL through the same
calls).  Checks the max-over-ranks time, the summed agent-steps and the stats all-reduce."""
import os
import sys
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))


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


def _bench(*args, timeout=300):
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(repo, "bench.py")] + list(args), env=env,
                         capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("world,total", [(2, 64), (3, 64)])
def test_bench_launcher_spawns_ranks(world, total):
    """bench.py --gpus N run directly starts N rank processes itself (the parent never touches the GPU):
    rank 0 prints one line with n_gpus N, the units summed over ranks over the max rank time, and the
    --total-envs split (configs[3]: 64 envs over the ranks) reduced over every rank."""
    line = _bench("--gpus", str(world), "--total-envs", str(total), "--launcher-selftest", "--backend", "gloo")
    assert line["n_gpus"] == world
    assert line["envs_total"] == total
    units = sum(100 * (r + 1) for r in range(world))
    assert abs(line["value"] - units / (0.01 * world)) < 1e-6


def test_bench_launcher_propagates_failure():
    """A rank that dies while the other waits in a collective: rank 1 exits 3 only after rank 0 has
    announced (rendezvous store) that it is entering a gloo barrier it can never leave.  The launcher
    must return non-zero well within the timeout and have terminated rank 0 (SIGTERM)."""
    import subprocess
    import sys
    import time
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t = time.time()
    out = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--launcher-selftest",
                          "--backend", "gloo", "--fail-rank", "1"], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 3, (out.returncode, out.stderr[-2000:])
    assert time.time() - t < 90
    assert "rank 1 exited 3" in out.stderr, out.stderr[-2000:]
    assert "rank 0 exited -15" in out.stderr, out.stderr[-2000:]     # stopped by the launcher, not finished


def test_cpu_baseline_uses_several_cores():
    """The CPU baseline runs one single-thread reference process per host core it is given and
    reports the aggregate with the core count."""
    import bench
    res = bench.run_cpu_baseline(1.0, 64, 256, procs=2)
    assert res is not None and res["cores"] == 2
    assert res["value"] > 0 and abs(res["per_core"] * 2 - res["value"]) < 1e-6
    use, shown = bench.host_cores()
    assert 1 <= use <= shown


def test_bench_refuses_more_rccl_ranks_than_gpus():
    """Under RCCL every rank needs its own GPU: a world above the device count fails loudly instead of
    wrapping ranks onto shared cards; gloo rehearsals wrap and report the GPUs actually spanned."""
    import bench
    assert bench.rank_device(8, 5, 8, "nccl") == (5, 8)
    assert bench.rank_device(1, 0, 1, "nccl") == (0, 1)
    with pytest.raises(RuntimeError, match="need 2 GPUs"):
        bench.rank_device(2, 1, 1, "nccl")
    assert bench.rank_device(2, 1, 1, "gloo") == (0, 1)
    assert bench.rank_device(3, 2, 2, "gloo") == (0, 2)
    with pytest.raises(RuntimeError):
        bench.rank_device(1, 0, 0, "nccl")


def _ising_worker(rank, world, port, R, T, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import numpy as np
    import ising_oracle
    from mfrl_amd.dist import reduce_ising, replica_block
    r0, n = replica_block(R, world, rank)
    res = [ising_oracle.mfq(16, 0.8, T, seed=13 + r0 + r) for r in range(n)]
    final = [x["order"][-1] for x in res]
    steps = np.array([x["steps"] for x in res])
    out[rank] = (r0, n, reduce_ising(final, steps), final)
    dist.destroy_process_group()


def test_two_rank_ising_replica_sharding():
    """Ising replicas over 2 gloo ranks (scripts/bench_ising.py --gpus 2): the blocks cover the replica range once
    (replica r on seed 13 + r wherever it runs), and the one all-reduce of (sum of final order parameters, sum of
    steps, replicas) equals the single-rank sum over the same replicas (main_MFQ_Ising.py:138-156's order
    parameter, here from the numpy oracle)."""
    import numpy as np
    import ising_oracle
    from mfrl_amd.dist import replica_block
    R, T, world = 7, 400, 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_ising_worker, args=(world, _free_port(), R, T, out), nprocs=world, join=True)
    blocks = sorted((out[r][0], out[r][1]) for r in range(world))
    assert blocks == [replica_block(R, world, r) for r in range(world)] == [(0, 4), (4, 3)]
    single = [ising_oracle.mfq(16, 0.8, T, seed=13 + r) for r in range(R)]
    want = [sum(x["order"][-1] for x in single), float(sum(x["steps"] for x in single)), float(R)]
    got = out[0][2]
    assert got == out[1][2]
    assert got[1:] == want[1:]
    assert abs(got[0] - want[0]) <= 1e-12 * max(1.0, abs(want[0]))
    finals = out[0][3] + out[1][3]
    assert np.array_equal(np.array(finals), np.array([x["order"][-1] for x in single]))
