"""Throughput bench: Battle 64x64, 256 agents -- agent-steps/s of the hot path (env.step + obs).

    python bench.py [--gpus N --steps K --warmup W] [--envs E] [--no-cpu-baseline]

Episodes are staggered over envs and the batch is run for one episode cap (400 steps) before
the warmup, so any K-step window sees the steady mix of episode phases (not just the opening
256-agent fight).  A *step* is one pass of the reference training-loop step (senario_battle.play :96-171) over
every env of the batch: get_observation for both groups (views + features written to HBM),
the synthetic rush policy of SURVEY.md 8(d) (on device), set_action, step (attack shuffle,
attacks, starve, moves, reward rules, done), get_reward, mean-action pooling, clear_dead,
and episode restart at done / 400 steps.  It is ONE kernel launch (k_rollout) per step.
`value` counts agents present at get_observation, summed over envs, steps and ranks, over the
max-over-ranks wall time of the K timed steps.  Multi-GPU: one process per GPU, each with its
own E envs (weak scaling); the only collective is the RCCL all-reduce of episode statistics.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd")
sys.path.insert(0, os.path.join(PKG, "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))

MAP, N_SIDE = 64, 128
BYTES_PER_AGENT_STEP = 4 * (1183 + 34) + 4 + 4 + 1 + 4 + 64      # 4,945 B
HBM_PEAK_GBS = 8000.0                                           # MI355X spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default 24576 at 64x64, 1024 at 256x256)")
    ap.add_argument("--map", type=int, default=MAP, help="map side (64: the metric's config; 256: configs[4])")
    ap.add_argument("--agents", type=int, default=2 * N_SIDE, help="agents per env, half per group")
    ap.add_argument("--max-steps", type=int, default=400)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--backend", default="nccl", help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.envs is None:
        # 64x64: 24576 envs per GPU -- a launch has a fixed cost (~0.15 ms: ramp-up and the tail of the
        # persistent grid), amortised over more envs: 16384 -> 24576 envs = +6-11 % agent-steps/s,
        # beyond ~28K the gain stops (profiles/r01_env_sweep.txt)
        a.envs = 24576 if a.map * a.map <= 64 * 64 else max(8, (16384 * 256) // a.agents)
    return a


# ----------------------------------------------------------------------------- CPU baseline
def cpu_baseline(seconds, map_size=MAP, n_side=N_SIDE):
    """Reference engine (oracle/_ref) if built, else the C oracle, single thread, same workload.

    Only env calls are timed (get_observation, get_agent_id, set_action, step, get_reward,
    get_alive, clear_dead) -- as in BASELINE.md; the numpy rush policy runs outside the clock."""
    import numpy as np
    import battle_driver as bd
    import magent
    ref = os.path.join(REPO, "oracle", "_ref", "libmagent_ref.so")
    port = os.path.join(REPO, "oracle", "build", "libbattle_oracle.so")
    path, kind = (ref, "reference") if os.path.exists(ref) else (port, "port")
    env = magent.GridWorld("battle", map_size=map_size, lib=magent.load_library(path))
    h = env.get_handles()
    _, v2a = env.get_view2attack(h[0])
    left, right = bd.block_positions(map_size, n_side)
    rng = np.random.RandomState(0)
    clock, agent_steps, episodes = 0.0, 0, 0
    while clock < seconds:
        t = time.perf_counter()
        env.reset()
        env.add_agents(h[0], method="custom", pos=left)
        env.add_agents(h[1], method="custom", pos=right)
        clock += time.perf_counter() - t
        done, k = False, 0
        while not done and k < 400 and clock < seconds:
            t = time.perf_counter()
            obs = [env.get_observation(h[g]) for g in range(2)]
            for g in range(2):
                env.get_agent_id(h[g])
            clock += time.perf_counter() - t
            acts = [bd.rush_policy(obs[g][0], obs[g][1], rng, v2a, 13, 21) for g in range(2)]
            t = time.perf_counter()
            for g in range(2):
                env.set_action(h[g], acts[g])
            done = env.step()
            for g in range(2):
                env.get_reward(h[g])
                env.get_alive(h[g])
            env.clear_dead()
            clock += time.perf_counter() - t
            agent_steps += len(obs[0][0]) + len(obs[1][0])
            k += 1
        episodes += 1
    return {"value": agent_steps / clock, "unit": "agent-steps/s", "cores": 1, "kind": kind,
            "sample": "%d agent-steps (%d episode starts) of Battle %dx%d/%d on 1 thread (OMP_NUM_THREADS=1), "
                      "%.1f s of timed env calls; %s" % (agent_steps, episodes, map_size, map_size, 2 * n_side, clock,
                                                         os.path.basename(path))}


def run_cpu_baseline_subprocess(seconds, map_size, agents):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-baseline-only",
                          "--cpu-seconds", str(seconds), "--map", str(map_size), "--agents", str(agents)],
                         env=env, capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        sys.stderr.write(out.stderr)
        return None
    return json.loads(out.stdout.strip().splitlines()[-1])


# ----------------------------------------------------------------------------- GPU bench
def main():
    args = parse()
    if args.cpu_baseline_only:
        print(json.dumps(cpu_baseline(args.cpu_seconds, args.map, args.agents // 2)))
        return
    import torch
    import torch.distributed as dist
    import battle_driver as bd
    from mfrl_amd.battle import BattleBatch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count())     # (rehearsals: several ranks on one GPU)
    torch.cuda.set_device(local)
    if world > 1:
        if args.backend == "nccl":           # RCCL over xGMI
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:                                # rehearsal of the N-rank flow without RCCL
            dist.init_process_group(args.backend)
    stream = torch.cuda.current_stream()

    eng = BattleBatch(args.map, args.envs, stream=stream)
    left, right = bd.block_positions(args.map, args.agents // 2)
    from mfrl_amd.dist import env_seed, reduce_stats, reduce_timing
    eng.rollout_init([left, right], max_steps=args.max_steps, eps=0.2, seed=env_seed(1234, rank))
    E = args.envs
    grid, _ = eng.rollout_info()
    big = grid == E and args.map * args.map > 64 * 64     # k_observe + k_rollout_big (state in HBM)
    steps_buf = torch.zeros(E, dtype=torch.int64, device="cuda")
    stats_buf = torch.zeros(E * 4, dtype=torch.float64, device="cuda")

    def agent_steps():
        eng.rollout_copy("agent_steps", steps_buf)
        return steps_buf.sum()

    # input preparation: run one episode cap of steps so that the staggered envs hold every
    # phase of an episode (early fights with ~256 agents ... late game with few survivors)
    eng.rollout_step(args.max_steps)
    for _ in range(args.warmup):
        eng.rollout_step(1)
    torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    a0 = agent_steps()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    red = None
    for k in range(args.steps):
        ev[k][0].record(stream)
        eng.rollout_step(1)
        ev[k][1].record(stream)
        # episode statistics -> RCCL all-reduce, once per episode batch (an episode cap of steps) and at
        # the end of the timed window: the only collective
        if world > 1 and ((k + 1) % args.max_steps == 0 or k == args.steps - 1):
            eng.rollout_copy("stats", stats_buf)
            red = reduce_stats(stats_buf.view(E, 4))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    a1 = agent_steps()
    if red is None:                  # one rank: the same statistics, reduced after the clock
        eng.rollout_copy("stats", stats_buf)
        red = reduce_stats(stats_buf.view(E, 4))
    red = red.tolist()
    kernel_ms = sum(s.elapsed_time(e) for s, e in ev) / args.steps
    local_units = float((a1 - a0).item())
    elapsed, total_units = reduce_timing(t1 - t0, local_units, "cuda")
    if rank == 0:
        ms_per_step = 1e3 * elapsed / args.steps
        units_per_launch = local_units / args.steps
        achieved = BYTES_PER_AGENT_STEP * units_per_launch / (kernel_ms * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(REPO, "profiles", "pmc_big256.json" if big else "pmc_k_rollout.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                pm = json.load(f)
            if pm.get("envs") == E and pm.get("map", MAP) == args.map:
                traffic = pm.get("hbm_bytes_per_launch", pm.get("hbm_bytes_per_step"))
        line = {
            "metric": "agent-steps/sec (env.step+obs) Battle %dx%dx%d agents" % (args.map, args.map, args.agents),
            "value": total_units / elapsed,
            "unit": "agent-steps/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (fixed-seed two-block placement, on-device rush policy)",
            "config": {"workload": "Battle %dx%d, %d+%d agents, %d envs per GPU, episode cap %d, %s"
                       % (args.map, args.map, args.agents // 2, args.agents // 2, E, args.max_steps,
                          "k_observe_items + k_rollout_big on 2 streams" if big else "fused step"),
                       "map": args.map, "agents": args.agents, "envs_per_gpu": E,
                       "parallelism": "envs sharded one process per GPU (dp%d)" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_observe_items+k_rollout_big" if big else "k_rollout", "kernel_ms": kernel_ms,
                         "bytes_per_unit": BYTES_PER_AGENT_STEP, "units_per_launch": units_per_launch},
            "cpu_baseline": None,
            "episodes": {"finished": red[0], "return_mean": [red[1] / max(red[0], 1.0), red[2] / max(red[0], 1.0)],
                         "kills": red[3], "note": "all ranks, since rollout_init (RCCL all-reduce per episode batch)"},
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = run_cpu_baseline_subprocess(args.cpu_seconds, args.map, args.agents)
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
