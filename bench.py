"""Throughput bench: Battle 64x64, 256 agents -- agent-steps/s of the hot path (env.step + obs).

    python bench.py [--gpus N --steps K --warmup W] [--envs E | --total-envs T] [--no-cpu-baseline]

Episodes are staggered over envs and the batch is run for one episode cap (400 steps) before
the warmup, so any K-step window sees the steady mix of episode phases (not just the opening
256-agent fight).  A *step* is one pass of the reference training-loop step (senario_battle.play :96-171) over
every env of the batch: get_observation for both groups (views + features written to HBM),
the synthetic rush policy of SURVEY.md 8(d) (on device), set_action, step (attack shuffle,
attacks, starve, moves, reward rules, done), get_reward, mean-action pooling, clear_dead,
and episode restart at done / 400 steps.  One k_rollout launch runs --substeps (default: the engine's choice, 20 here) such
steps of every env back to back while the env's image stays in LDS, for 131072 envs per GPU; the timed
region is exactly K steps (ceil(K / substeps) launches, the last one the remainder), bit-identical to K
one-step launches.
`value` counts agents present at get_observation, summed over envs, steps and ranks, over the
max-over-ranks wall time of the K timed steps.

Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) this process is one
rank; run directly with --gpus N > 1 it starts N fresh rank processes itself (before anything here
touches the GPU) and exits with their status.  --envs E: E envs per rank (weak scaling);
--total-envs T: T envs split over the ranks (strong scaling, configs[3]: 64 envs over 8 GPUs).
The only collective is the RCCL all-reduce of the episode statistics.

Self-check (after the clock, outside the timed region): every rank replays --check-envs sampled envs of
its own batch on the C oracle from rollout_init on (tests/rollout_check.py: the oracle steps with a host
restatement of the device's counter-hash rush policy) and compares the last step's observation, actions,
rewards and mean action, the state after it (ids, positions, hp), and the env's counters (agent-steps,
episode statistics, running return) bit for bit; it also reads the device and queue error words
(rollout_check).  The line's "check" records it; a mismatch exits non-zero.
"""
import argparse
import hashlib
import json
import os
import socket
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
LIB = os.path.join(PKG, "build", "libmagent.so")


def lib_sha16(path=LIB):
    """Content hash of the engine library: the key under which PMC counters of a build are filed (a counter file
    of another build is never attached to this build's line)."""
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def measure_ceiling(eng, total_bytes, reps=2):
    """The HBM write ceiling of this GPU, measured in this process after the clock (report a
    measured stream peak beside the nominal one): a write-only float4 stream of the same byte count as one timed
    launch's algorithmic bytes over the same view buffer, in each store shape of BattleBatch.STORE_SHAPES, best
    of `reps` per shape.  None when the buffer is too small to leave the caches (few envs)."""
    import ctypes
    ptr, n = ctypes.c_void_p(), ctypes.c_size_t()
    eng._check(eng._dll.mfx_battle_rollout_buffer(eng.game, b"view", 0, ctypes.byref(ptr), ctypes.byref(n)),
               "rollout_buffer")
    if n.value < (1 << 30):
        return None
    total = max(int(total_bytes), n.value, 16 << 30)
    best = [0.0] * len(eng.STORE_SHAPES)
    for _ in range(reps):
        for sh in range(len(best)):
            best[sh] = max(best[sh], eng.store_ceiling(total, sh))
    k = max(range(len(best)), key=lambda i: best[i])
    return {"peak": best[k], "shape": eng.STORE_SHAPES[k], "bytes": total, "region_bytes": n.value,
            "per_shape_gbs": dict(zip(eng.STORE_SHAPES, best)),
            "what": "write-only float4 stream (mfx_store_ceiling, csrc/diag_kernels.hip) of the timed launch's "
                    "algorithmic bytes over the same view buffer, same process and GPU, after the clock; best of "
                    "%d per shape" % reps}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default 131072 at 64x64, 2048 at 256x256)")
    ap.add_argument("--total-envs", type=int, default=None,
                    help="envs over all GPUs, split evenly (strong scaling; configs[3]: --total-envs 64)")
    ap.add_argument("--map", type=int, default=MAP, help="map side (64: the metric's config; 256: configs[4])")
    ap.add_argument("--agents", type=int, default=2 * N_SIDE, help="agents per env, half per group")
    ap.add_argument("--max-steps", type=int, default=400)
    # 20 consecutive steps of every env per launch (env image kept in LDS between them on k_rollout): the
    # launch ramp-up / tail and the env install / write-back are paid once per 20 steps.  At the round-2
    # batch of 49152 envs 4 steps gained 9-11 % over one and 8 little more (profiles/r02_substeps_sweep.txt);
    # with 131072 envs 8 steps gain 3-4 % over 4 (profiles/r03_env_sweep.txt) and 20 another 3-4 % over 8
    # (profiles/r03_substeps20.txt).  The queue kernel k_rollout_bigq (256x256 envs, and batches of few
    # 64x64 envs): 20 steps per launch, +0.3 % over 16 at 60 steps, +1-2 % at 20 steps (one launch, not
    # 16 + 4).  The results are bit-identical for any value
    # (tests/test_rollout_gpu.py::test_rollout_substeps_match_single_steps); the engine takes 1..64, and 0 lets it
    # choose per path and batch (BattleEngine::sub_steps, profiles/r04_substeps_auto.txt): 20 here at 131072 envs
    # and at 256x256, 2 for k_rollout below 96 envs per CU (8192 envs: 0.556 -> 0.594), and for the pipelined
    # few-env stepper the whole timed region as one launch (8 envs: 0.0356 ms per step at 20, 0.0285 at 64).
    ap.add_argument("--substeps", type=int, default=0,
                    help="consecutive steps of every env per launch (default 0: the engine's choice, 20 at the default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-procs", type=int, default=None,
                    help="concurrent single-thread CPU-baseline processes (default: the host cores this job may use)")
    ap.add_argument("--cpu-seed", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--backend", default="nccl", help=argparse.SUPPRESS)
    ap.add_argument("--launcher-selftest", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--fail-rank", type=int, default=-1, help=argparse.SUPPRESS)   # launcher self-test only
    ap.add_argument("--policy", choices=("rush", "qnet", "mfac"), default="rush",
                    help="rush: the on-device synthetic policy (the metric); qnet: two random-init mean-field Q "
                         "networks (ValueNet, algo/base.py:123-183) on the HIP forward, one per group; mfac: two "
                         "random-init MFAC actor-critic networks (algo/ac.py:219-276) on the HIP forward + draw")
    ap.add_argument("--no-ceiling", dest="ceiling", action="store_false",
                    help="skip the measured write ceiling after the clock (roofline.measured_peak)")
    ap.add_argument("--split", type=int, default=None,
                    help="the envs as this many engines on their own HIP streams, so one engine's launch overlaps "
                         "another's (default: rush 2 for 64x64 batches of 2048-16384 envs per GPU -- the launch tails "
                         "at under 16 envs per workgroup: 8192 envs 0.60 -> 0.67-0.87 by box, 16384 0.64 -> 0.73, "
                         "profiles/r06_split.txt -- else 1; mfac 2 -- 1.016e8 -> 1.051e8 agent-steps/s, "
                         "profiles/r06_mfac.txt; qnet 1)")
    ap.add_argument("--dense-view", action="store_true",
                    help="mfac: the view layer over all 1,183 inputs (A/B; default: the engine's view support)")
    ap.add_argument("--check-envs", type=int, default=8,
                    help="envs per rank replayed on the C oracle after the timed region (0: no check)")
    a = ap.parse_args(argv)
    if a.envs is None and a.total_envs is None and a.policy != "rush":
        a.envs = 8192                 # the network forward bounds these modes (1.2 / 3.4 MFLOP per agent-step)
    if a.split is None and a.policy != "rush":
        a.split = 2                   # one engine's env step under the other's forward (qnet 3.33 -> 3.38e7, r06_qnet_split.txt)
    if a.envs is None and a.total_envs is None:
        # 64x64: 131072 envs per GPU (~160 GB of observation buffers, 56 % of the HBM) -- a launch has a fixed
        # cost (ramp-up and the tail of the persistent grid: the last env of each of 1280 workgroups), amortised
        # over more envs per workgroup: at 8 steps per launch 49152 -> 65536 -> 98304 -> 131072 envs =
        # 1.19 -> 1.25 -> 1.30 -> 1.31-1.32e9 agent-steps/s, same box (profiles/r03_env_sweep.txt; round 2 at 4
        # steps: 24576 -> 49152 = 1.09 -> 1.146e9, profiles/r02_env_sub_sweep.txt)
        # 256x256 (4096 agents): 2048 envs (40 GB of observation buffers) -- 1024 -> 2048 envs at 16 steps per
        # k_rollout_bigq launch = 1.21-1.22 -> 1.27-1.29e9 (frac 0.75 -> 0.79-0.80), 3072 loses (0.68)
        # (profiles/r03_env_sweep256.txt)
        a.envs = 131072 if a.map * a.map <= 64 * 64 else max(8, (32768 * 256) // a.agents)
    return a


def rank_device(world, local, device_count, backend):
    """(device index of this rank, GPUs the job spans).  RCCL ("nccl") needs one GPU per rank: a world larger
    than the node's device count is refused, not wrapped onto shared cards.  Other backends (gloo rehearsals
    of the N-rank flow on one card) wrap local ranks over the devices, and the line reports the GPUs they
    actually span beside the rank count."""
    if device_count < 1:
        raise RuntimeError("bench.py: no GPU visible")
    if backend == "nccl" and world > device_count:
        raise RuntimeError("bench.py: %d ranks over RCCL need %d GPUs, this node shows %d (ranks never share a GPU "
                           "under RCCL; rehearse with --backend gloo)" % (world, world, device_count))
    return local % device_count, min(world, device_count)


class _StdoutToStderr:
    """fd 1 -> fd 2 while the process group initialises: the gloo library prints its connection messages on
    stdout from C++, and the bench's stdout must carry exactly one JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def rank_envs(args, world, rank):
    """Envs this rank steps: --envs per rank, or its share of --total-envs (remainder to low ranks)."""
    if args.total_envs is None:
        return args.envs
    return args.total_envs // world + (1 if rank < args.total_envs % world else 0)


# ----------------------------------------------------------------------------- N-rank launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n, argv, script=None):
    """Start n rank processes of this script -- or of `script` (scripts/bench_ising.py shares the launcher) --
    (torch.distributed.run's env contract, 127.0.0.1 rendezvous) and wait for them.  Called before anything in this process touches the GPU; the
    ranks are fresh children, so no GPU context is ever inherited or exec'd over.  If one rank
    fails the others are stopped (they would wait at a barrier).  Returns the worst exit status."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(script or __file__)] + list(argv), env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0:
                status = status or rc
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    if status:
        for r, p in enumerate(procs):
            sys.stderr.write("bench launcher: rank %d exited %d\n" % (r, p.returncode))
    return status


def launcher_selftest(args):
    """One rank of the launcher rehearsal (CPU, gloo): the same rank/env handling and reductions as the
    GPU bench, without the engine.  Rank r 'processes' 100*(r+1) units in 0.01*(r+1) s."""
    import torch
    import torch.distributed as dist
    from mfrl_amd.dist import reduce_stats, reduce_timing
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        with _StdoutToStderr():
            dist.init_process_group("gloo")
    if world > 1 and args.fail_rank >= 0:
        # a rank that dies while the others wait in a collective: rank fail_rank exits 3 once every other
        # rank has announced (through the rendezvous store) that it is entering the barrier
        store = dist.distributed_c10d._get_default_store()
        if rank == args.fail_rank:
            store.wait(["entering%d" % r for r in range(world) if r != rank])
            time.sleep(0.3)
            os._exit(3)
        store.set("entering%d" % rank, "1")
        dist.barrier()                       # never completes: the launcher must stop this rank
        return
    E = rank_envs(args, world, rank)
    red = reduce_stats(torch.ones(E, 4, dtype=torch.float64)).tolist()
    elapsed, units = reduce_timing(0.01 * (rank + 1), 100 * (rank + 1), "cpu")
    if rank == 0:
        print(json.dumps({"n_gpus": world, "value": units / elapsed, "envs_total": red[0], "elapsed": elapsed}))
    if world > 1:
        dist.destroy_process_group()


# ----------------------------------------------------------------------------- CPU baseline
def cpu_baseline(seconds, map_size=MAP, n_side=N_SIDE, seed=0):
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
    rng = np.random.RandomState(seed)
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
    return {"value": agent_steps / clock, "agent_steps": agent_steps, "episodes": episodes, "clock": clock,
            "kind": kind, "lib": os.path.basename(path)}


def host_cores():
    """(cores this job may use, cores the host shows).  On the GPU box `nproc` shows the whole
    machine while one GPU's job gets a share of it (OMP_NUM_THREADS is set to that share there)."""
    try:
        shown = len(os.sched_getaffinity(0))
    except AttributeError:
        shown = os.cpu_count() or 1
    share = os.environ.get("MFX_CPU_SHARE") or os.environ.get("OMP_NUM_THREADS")
    use = min(shown, int(share)) if share and share.isdigit() and int(share) > 0 else shown
    return max(1, use), shown


def run_cpu_baseline(seconds, map_size, agents, procs=None):
    """P concurrent single-thread reference-engine processes (OMP_NUM_THREADS=1: the reference attack
    loop is racy with more threads, GridWorld.cc:522), one per host core of this job, each on its own
    policy seed.  value = the sum of their rates (they run side by side for the same time)."""
    use, shown = host_cores()
    P = procs or use
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", "--cpu-seconds", str(seconds),
           "--map", str(map_size), "--agents", str(agents)]
    ps = [subprocess.Popen(cmd + ["--cpu-seed", str(i)], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True) for i in range(P)]
    res = []
    for p in ps:
        out, err = p.communicate(timeout=600)
        if p.returncode != 0:
            sys.stderr.write(err)
            return None
        res.append(json.loads(out.strip().splitlines()[-1]))
    total = sum(r["value"] for r in res)
    steps = sum(r["agent_steps"] for r in res)
    return {"value": total, "unit": "agent-steps/s", "cores": P, "kind": res[0]["kind"],
            "per_core": total / P, "host_nproc": shown,
            "whole_host_estimate": total / P * shown,      # per_core x every host core (linear: no shared state)
            "sample": "%d concurrent single-thread processes (OMP_NUM_THREADS=1), each %.0f s of timed env calls "
                      "of Battle %dx%d/%d (rush policy outside the clock): %d agent-steps, %d episode starts in "
                      "total; %s" % (P, seconds, map_size, map_size, agents, steps, sum(r["episodes"] for r in res),
                                     res[0]["lib"])}


# ----------------------------------------------------------------------------- self-check
def run_check(engs, args, sizes, placement, seeds, world):
    """Replay args.check_envs sampled envs of this rank's batch (spread over its engines) on the C oracle from
    rollout_init through the preparation, warmup and timed steps (tests/rollout_check.py), one of them on the
    reference engine itself as well; all ranks' verdicts reduced."""
    if args.check_envs <= 0:
        return None
    import torch
    import torch.distributed as dist
    import rollout_check as rc
    steps = args.max_steps + args.warmup + args.steps            # every step since rollout_init
    ref_lib = os.path.join(REPO, "oracle", "_ref", "libmagent_ref.so")
    t = time.perf_counter()
    err = None
    bad, sample, ref_env = [], [], None
    H = len(engs)
    for h, (eng, E, seed) in enumerate(zip(engs, sizes, seeds)):
        envs = rc.sample_envs(E, max(1, args.check_envs // H + (1 if h < args.check_envs % H else 0)))
        sample.append(envs)
        try:
            chk = rc.RolloutChecker(eng, args.map, placement, envs, args.max_steps, True, seed, 0.2)
            bad += [("engine %d: " % h if H > 1 else "") + b for b in chk.check(steps)]
            if h == 0 and os.path.exists(ref_lib):
                # one of the sampled envs replayed on the reference engine itself as well
                ref_env = envs[len(envs) // 2]
                ref = rc.RolloutChecker(eng, args.map, placement, [ref_env], args.max_steps, True, seed, 0.2,
                                        lib=ref_lib)
                bad += ["reference build: " + b for b in ref.check(steps)]
        except Exception as x:              # a device / queue error word (rollout_check) or a failed read
            bad, err = bad + ["%s: %s" % (type(x).__name__, x)], True
    n_local = sum(len(x) for x in sample)
    ok = torch.tensor([0.0 if bad else 1.0], dtype=torch.float64, device="cuda")
    n = torch.tensor([float(n_local)], dtype=torch.float64, device="cuda")
    nref = torch.tensor([0.0 if ref_env is None else 1.0], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        dist.all_reduce(n)
        dist.all_reduce(nref)
    return {"ok": bool(ok.item() == 1.0), "envs": int(n.item()), "envs_per_rank": n_local, "steps": steps,
            "sample_rank0": sample[0] if H == 1 else sample, "path": engs[0].rollout_path() if err is None else None,
            "reference_envs": int(nref.item()), "reference_env_rank0": ref_env,
            "what": "each sampled env replayed from rollout_init on the C oracle (oracle/battle_oracle.c) with a "
                    "host restatement of the device rush policy, and one of them (reference_env_rank0) also on the "
                    "reference engine itself (oracle/_ref, built from /root/reference); last step's views, features, "
                    "actions, rewards, mean action, post-step ids / positions (/ hp on the C oracle), agent-steps, "
                    "episode statistics and return compared bit for bit; device and queue error words read "
                    "(rollout_check); after the clock",
            "seconds": time.perf_counter() - t, "mismatches": bad[:16]}


# ----------------------------------------------------------------------------- learned policy
QNET_FLOP_PER_AGENT = 2 * (121 * 32 * 63 + 81 * 32 * 288 + 2592 * 256 + 34 * 32 + 21 * 64 + 64 * 32 + 320 * 128 +
                           128 * 64 + 64 * 21)          # 3,417,920: the mean-field QNet forward of one agent
ACNET_FLOP_PER_AGENT = 2 * (1183 * 256 + 34 * 256 + 512 * 512 + 512 * 21)   # 1,168,896: the AC / MFAC policy path
F32_MFMA_PEAK_TFS = 157.3                               # MI355X_MICROARCH.md (f32-input MFMA = the f32 VALU rate)


def main_qnet(args):
    """One process, one GPU: a learned policy in the loop (--policy qnet / mfac).  Per step: the HIP forward
    of each group's model on the observation in the rollout buffers (mfx_qnet_act_rollout: greedy Q;
    mfx_acnet_act_rollout: the MFAC policy and its draw), then one k_rollout launch that acts with those actions,
    steps and observes (mfx_battle_rollout_policy_step).  Random-init networks (torch modules, packed once); the
    value counts agent-steps as the rush line does.  The roofline is the forward's: f32 MFMA FLOPs (the MFMAs the
    kernels execute) over the two forwards' HIP-event time.

    --split H: the envs as H engines of E / H envs, each stepping on its own HIP stream with the same networks, so
    one engine's env step (k_rollout: HBM-bound observation writes) runs while another's forward (MFMA) does --
    the loop of senario_battle.play (:96-171) on H independent env batches.  mfac: the view layer runs over the
    inputs the engine's observation can make non-zero (BattleBatch.view_support, bit-identical, --dense-view: off).
    After the clock the same steps run once more with every engine on one stream and HIP events around each
    phase: the line's kernel_ms (forward) and env_step_ms (k_rollout) per step, serialised."""
    import torch
    import battle_driver as bd
    from mfrl_amd.algo.nets import ACNet, QNet
    from mfrl_amd.battle import BattleBatch
    from mfrl_amd.policy import ACNetHIP, QNetHIP
    torch.cuda.set_device(0)
    E = args.envs if args.total_envs is None else args.total_envs
    H = max(1, min(args.split, E))
    sizes = [E // H + (1 if h < E % H else 0) for h in range(H)]
    main = torch.cuda.current_stream()
    streams = [main] + [torch.cuda.Stream() for _ in range(H - 1)]
    left, right = bd.block_positions(args.map, args.agents // 2)
    os.environ.setdefault("MFX_SMALL_E", "0")                # (the fused k_rollout path at any E)
    engs = []
    for h in range(H):
        eng = BattleBatch(args.map, sizes[h], stream=streams[h])
        eng.rollout_init([left, right], max_steps=args.max_steps, eps=0.0, seed=1234 + 7919 * h)
        engs.append(eng)
    torch.manual_seed(7)
    pols = []
    ac = args.policy == "mfac"
    for g in range(2):
        if ac:
            pols.append(ACNetHIP((13, 13, 7), (34,), 21, True).load(ACNet((13, 13, 7), (34,), 21, use_mf=True).cuda()))
        else:
            pols.append(QNet((13, 13, 7), (34,), 21, True).cuda())
    # ACNetHIP keeps its row lists per engine; a QNetHIP handle owns one conv-activation scratch, so each engine gets
    # its own pair of handles over the same weights (--split)
    pol_of = [pols] * H if ac else [[QNetHIP((13, 13, 7), (34,), 21, True).load(pols[g]) for g in range(2)]
                                     for _ in range(H)]
    torch.cuda.synchronize()
    support = ac and not args.dense_view
    step_no = [0]
    steps_buf = [torch.zeros(n, dtype=torch.int64, device="cuda") for n in sizes]

    def agent_steps():
        tot = torch.zeros((), dtype=torch.int64, device="cuda")
        for h, eng in enumerate(engs):
            eng.rollout_copy("agent_steps", steps_buf[h])
            eng.sync()
            tot += steps_buf[h].sum()
        return tot

    def act(h):
        for g in range(2):
            if ac:
                pol_of[h][g].act_rollout(engs[h], g, 1234 + 7919 * h, step_no[0], support=support)
            else:
                pol_of[h][g].act_rollout(engs[h], g)

    def one_step():
        for h, eng in enumerate(engs):
            with torch.cuda.stream(streams[h]):
                act(h)
                eng.rollout_policy_step()
        step_no[0] += 1

    for h, eng in enumerate(engs):
        with torch.cuda.stream(streams[h]):
            eng.rollout_policy_observe()
    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    a0 = agent_steps()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    units = float((agent_steps() - a0).item())
    # the phases, serialised: every engine on the main stream, events around each engine's forwards and step
    n_ph = max(1, min(args.steps, 6))
    evs = []
    for h, eng in enumerate(engs):
        eng.set_stream(main)
    for k in range(n_ph):
        for h, eng in enumerate(engs):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(main)
            act(h)
            e[1].record(main)
            eng.rollout_policy_step()
            e[2].record(main)
            evs.append(e)
        step_no[0] += 1
    torch.cuda.synchronize()
    fwd_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / n_ph
    env_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / n_ph
    for eng in engs:
        eng.rollout_check()
    units_step = units / args.steps
    if ac:
        kv = pol_of[0][0].input_support_size() or 1183
        flop_dense = ACNET_FLOP_PER_AGENT
        flop_per_agent = 2 * (kv * 256 + 34 * 256 + 512 * 512 + 512 * 21)
    else:
        flop_dense = flop_per_agent = QNET_FLOP_PER_AGENT
    flops = flop_per_agent * units_step
    what = ("learned MFAC policy (HIP actor-critic forward + draw)" if ac else
            "learned MF-Q policy (HIP QNet forward)")
    line = {"metric": "agent-steps/sec (env.step+obs) Battle %dx%dx%d agents, %s" % (args.map, args.map, args.agents,
                                                                                     what),
            "value": units / (t1 - t0), "unit": "agent-steps/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * (t1 - t0) / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic (random-init networks)",
            "config": {"workload": "Battle %dx%d, %d envs, two %s (one per group), forward + fused step per step%s"
                                   % (args.map, args.map, E, "MFAC networks" if ac else "mean-field QNets",
                                      "; the envs as %d engines on %d HIP streams" % (H, H) if H > 1 else ""),
                       "envs_per_gpu": E, "policy": args.policy, "engines": H,
                       "view_inputs": (pols[0].input_support_size() or 1183) if ac else 1183},
            "roofline": {"bound": "mfma", "achieved": flops / (fwd_ms * 1e-3) / 1e12, "peak": F32_MFMA_PEAK_TFS,
                         "unit": "TFLOP/s", "frac": flops / (fwd_ms * 1e-3) / 1e12 / F32_MFMA_PEAK_TFS,
                         "traffic": None, "kernel": "k_acnet (x2 groups)" if ac else "k_qnet_conv + k_qnet_head (x2 groups)",
                         "kernel_ms": fwd_ms, "env_step_ms": env_ms,
                         "kernel_ms_is": "the forwards (both groups, every engine) of one step, serialised after the "
                                         "clock on one stream (HIP events; mean of %d steps); env_step_ms: the k_rollout "
                                         "step + observation of every engine the same way" % n_ph,
                         "flop_per_unit": flop_per_agent, "flop_per_unit_dense": flop_dense,
                         "flop_is": "the MFMA FLOPs executed per agent (the view layer over the inputs the "
                                    "observation can make non-zero when view_inputs < 1183); flop_per_unit_dense: the "
                                    "dense network's",
                         "units_per_step": units_step}}
    print(json.dumps(line), flush=True)
    return 0


# ----------------------------------------------------------------------------- GPU bench
def main():
    args = parse()
    if args.cpu_baseline_only:
        print(json.dumps(cpu_baseline(args.cpu_seconds, args.map, args.agents // 2, seed=args.cpu_seed)))
        return 0
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    if args.launcher_selftest:
        launcher_selftest(args)
        return 0
    if args.policy != "rush":
        return main_qnet(args)
    import torch
    import torch.distributed as dist
    import battle_driver as bd
    from mfrl_amd.battle import BattleBatch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local, n_gpus = rank_device(world, int(os.environ.get("LOCAL_RANK", "0")), torch.cuda.device_count(),
                                args.backend if world > 1 else "nccl")
    torch.cuda.set_device(local)
    if world > 1:
        if args.backend == "nccl":           # RCCL over xGMI
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:                                # rehearsal of the N-rank flow without RCCL
            with _StdoutToStderr():
                dist.init_process_group(args.backend)
    E = rank_envs(args, world, rank)
    # (ranks sharing a card -- the gloo rehearsal -- run the same kernels as one rank per GPU: the queue kernels
    # complete with one resident workgroup per XCD, DESIGN.md §5 "Forward progress")
    stream = torch.cuda.current_stream()
    left, right = bd.block_positions(args.map, args.agents // 2)
    from mfrl_amd.dist import env_seed, reduce_stats, reduce_timing
    # the envs as H engines on H HIP streams (--split; default: 2 for k_rollout batches of under 16 envs per
    # workgroup): one engine's launch tail runs beside the other's launch (profiles/r06_split.txt)
    H = args.split if args.split is not None else (
        2 if args.map * args.map <= 64 * 64 and 2048 <= E <= 16384 and args.policy == "rush" else 1)
    H = max(1, min(H, E))
    sizes = [E // H + (1 if h < E % H else 0) for h in range(H)]
    streams = [stream] + [torch.cuda.Stream() for _ in range(H - 1)]
    seeds = [env_seed(1234, rank) + 104729 * h for h in range(H)]
    engs = []
    for h in range(H):
        e = BattleBatch(args.map, sizes[h], stream=streams[h])
        e.rollout_init([left, right], max_steps=args.max_steps, eps=0.2, seed=seeds[h])
        e.rollout_substeps(max(0, args.substeps))
        engs.append(e)
    eng = engs[0]
    path = eng.rollout_path()               # the kernels rollout_step runs (chosen by the engine)
    grid, lds = eng.rollout_info()          # persistent grid, LDS bytes per workgroup
    S = eng.get_substeps()                  # (0: the engine's choice for this path and batch)
    big = path in ("k_rollout_bigq", "k_observe_items+k_rollout_big")   # large envs, state in HBM
    steps_buf = [torch.zeros(n, dtype=torch.int64, device="cuda") for n in sizes]
    stats_buf = [torch.zeros(n * 4, dtype=torch.float64, device="cuda") for n in sizes]

    def join():                             # the main stream waits for every engine's stream
        for st in streams[1:]:
            ev = torch.cuda.Event()
            ev.record(st)
            stream.wait_event(ev)

    def fork():                             # every engine's stream waits for the main stream
        ev = torch.cuda.Event()
        ev.record(stream)
        for st in streams[1:]:
            st.wait_event(ev)

    def agent_steps():
        for e, b in zip(engs, steps_buf):
            e.rollout_copy("agent_steps", b)
        join()
        return sum(b.sum() for b in steps_buf)

    def stats():
        for e, b in zip(engs, stats_buf):
            e.rollout_copy("stats", b)
        join()
        return torch.cat(stats_buf).view(E, 4)

    # input preparation: run one episode cap of steps so that the staggered envs hold every
    # phase of an episode (early fights with ~256 agents ... late game with few survivors)
    for e in engs:
        e.rollout_step(args.max_steps + args.warmup)
    torch.cuda.synchronize()

    # launches of the timed region: S steps each (the last one the remainder); HIP events on the main stream around
    # the whole region, the engines' streams forked from and joined into it (an event pair around every launch put
    # two timestamp packets between consecutive launches: at 8192 envs x 2 steps per launch ~5 % of the wall time)
    chunks = [min(S, args.steps - k) for k in range(0, args.steps, S)]
    # one event pair per run of launches between collectives (one run at world 1): the roofline's kernel time
    # leaves the statistics' all-reduce and the wait for other ranks out
    segs = []
    a0 = agent_steps()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    red = None
    done_steps = 0
    for k, n in enumerate(chunks):
        if not segs or segs[-1][1] is not None:
            segs.append([torch.cuda.Event(enable_timing=True), None])
            segs[-1][0].record(stream)
            fork()
        for e in engs:
            e.rollout_step(n)
        done_steps += n
        # episode statistics -> RCCL all-reduce, once per episode batch (an episode cap of steps) and at
        # the end of the timed window: the only collective
        if world > 1 and (done_steps // args.max_steps != (done_steps - n) // args.max_steps or k == len(chunks) - 1):
            join()
            segs[-1][1] = torch.cuda.Event(enable_timing=True)
            segs[-1][1].record(stream)
            red = reduce_stats(stats())
    if segs[-1][1] is None:
        join()
        segs[-1][1] = torch.cuda.Event(enable_timing=True)
        segs[-1][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    a1 = agent_steps()
    if red is None:                  # one rank: the same statistics, reduced after the clock
        red = reduce_stats(stats())
    red = red.tolist()
    # the mean launch (round of H concurrent launches) of the timed region: the runs' time / their launch count
    kernel_ms = sum(a.elapsed_time(b) for a, b in segs) / len(chunks)
    local_units = float((a1 - a0).item())
    elapsed, total_units = reduce_timing(t1 - t0, local_units, "cuda")
    check = run_check(engs, args, sizes, [left, right], seeds, world)
    # the measured write ceiling of this GPU (after the check: it overwrites the view buffer)
    ceiling = measure_ceiling(eng, BYTES_PER_AGENT_STEP * local_units / len(chunks)) if args.ceiling else None
    if rank == 0:
        ms_per_step = 1e3 * elapsed / args.steps
        steps_per_timed_launch = args.steps / len(chunks)       # the mean launch kernel_ms is
        S_run = max(chunks)                  # the launches of the timed region (S caps them at K steps)
        units_per_launch = local_units / len(chunks)
        achieved = BYTES_PER_AGENT_STEP * units_per_launch / (kernel_ms * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(REPO, "profiles", "pmc_big256.json" if big else "pmc_k_rollout.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                pm = json.load(f)
            # counters are attached only when they were collected on this build of the library at this shape
            if (pm.get("envs") == E and pm.get("map", MAP) == args.map and pm.get("substeps", 1) == S
                    and pm.get("engines", 1) == H and pm.get("lib_sha16") == lib_sha16()):
                traffic = pm.get("hbm_bytes_per_launch", pm.get("hbm_bytes_per_step"))
        strong = args.total_envs is not None
        kern = {"k_rollout_obs+k_rollout": "k_rollout"}.get(path, path)
        line = {
            "metric": "agent-steps/sec (env.step+obs) Battle %dx%dx%d agents" % (args.map, args.map, args.agents),
            "value": total_units / elapsed,
            "unit": "agent-steps/s",
            "n_gpus": n_gpus, "ranks": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (fixed-seed two-block placement, on-device rush policy)",
            "config": {"workload": "Battle %dx%d, %d+%d agents, %s, episode cap %d, %s"
                       % (args.map, args.map, args.agents // 2, args.agents // 2,
                          (("%d envs over %d GPUs" % (args.total_envs, world)) if n_gpus == world else
                           ("%d envs over %d ranks on %d GPU(s)" % (args.total_envs, world, n_gpus))) if strong else
                          "%d envs per GPU" % E if n_gpus == world else "%d envs per rank" % E,
                          args.max_steps,
                          (("%s, %d steps per launch" % (path, S_run)) if big else
                           ("fused step" if S_run == 1 else "fused step, %d consecutive steps per launch" % S_run)) +
                          ("; the envs as %d engines of %s envs on %d HIP streams" % (H, "/".join(map(str, sorted(set(sizes)))), H)
                           if H > 1 else "")),
                       "map": args.map, "agents": args.agents, "envs_per_gpu": E, "steps_per_launch": S_run,
                       "engines": H,
                       # agents placed per episode start vs the live agents an env-step actually carries (the
                       # unit counts live agents; battles thin the armies, staggered episodes mix all phases)
                       "live_agents_per_env_step": local_units / (args.steps * E),
                       "parallelism": ("envs sharded one process per GPU (dp%d)" % world) if n_gpus == world else
                                      ("%d ranks on %d GPU(s), %s rehearsal" % (world, n_gpus, args.backend))},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": kern, "kernel_ms": kernel_ms,
                         "kernel_ms_is": "mean launch duration: HIP events on the launch stream around the timed "
                                         "region's %d launch(es) (%d run(s) of back-to-back launches between "
                                         "collectives), / their count; %g step(s) per launch%s"
                                         % (len(chunks), len(segs), steps_per_timed_launch,
                                            "; each launch here is %d concurrent launches, one per engine and stream "
                                            "(the events on the main stream, the engines' streams forked from and "
                                            "joined into it)" % H if H > 1 else ""),
                         "bytes_per_unit": BYTES_PER_AGENT_STEP, "units_per_launch": units_per_launch,
                         "measured_peak": ceiling["peak"] if ceiling else None,
                         "frac_measured": achieved / ceiling["peak"] if ceiling else None,
                         "measured_peak_detail": ceiling,
                         "traffic_is": ("HBM bytes per launch from rocprofv3 FETCH_SIZE (x2, gfx950) and WRITE_SIZE "
                                        "passes of this library build (lib_sha16 %s), %s" % (lib_sha16(), pmc))
                                       if traffic is not None else
                                       "null: no counter file of this library build (lib_sha16 %s) at this shape"
                                       % lib_sha16(),
                         "grid": grid, "lds_bytes": lds},
            "cpu_baseline": None,
            "episodes": {"finished": red[0], "return_mean": [red[1] / max(red[0], 1.0), red[2] / max(red[0], 1.0)],
                         "kills": red[3],
                         "note": "all ranks, since rollout_init (%s)" % (
                             "one rank: reduced locally after the clock" if world == 1 else
                             "RCCL all-reduce over xGMI per episode batch" if args.backend == "nccl" else
                             "%s all-reduce per episode batch: a rehearsal of the N-rank flow, not RCCL" % args.backend)},
        }
        if check is not None:
            line["check"] = check
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = run_cpu_baseline(args.cpu_seconds, args.map, args.agents, args.cpu_procs)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if check is not None and not check["ok"]:
        sys.stderr.write("bench self-check FAILED: %s\n" % check["mismatches"][:8])
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
