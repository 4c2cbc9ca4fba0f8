"""Self-play training, train_battle.py (reference root) without TensorFlow.

    python -m mfrl_amd.train_battle --algo mfq --n_round 2000 --map_size 40 --max_steps 400
    python -m mfrl_amd.train_battle --algo mfq --envs 256 ...     # batched engine, all in HBM

Same arguments, epsilon schedule (linear_decay) and Runner as the reference; models from
mfrl_amd.algo (PyTorch-ROCm), the env from the drop-in magent (one env) or a BattleBatch (--envs).
Logs go to data/tmp/<algo>.jsonl, models to data/models/<algo>-{0,1}/<algo>_<round>.pt.
"""
import argparse
import os
import time

import torch

import magent

from .algo import spawn_ai, tools
from .algo.play import play, play_batched


def linear_decay(epoch, x, y):
    """train_battle.py:15-35: piecewise-linear interpolation of y over the breakpoints x."""
    min_v = y[0]
    start = x[0]
    if epoch == start:
        return min_v
    eps = min_v
    for i, x_i in enumerate(x):
        if epoch <= x_i:
            interval = (y[i] - y[i - 1]) / (x_i - x[i - 1])
            eps = interval * (epoch - x[i - 1]) + y[i - 1]
            break
    return eps


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--algo", type=str, choices={"ac", "mfac", "mfq", "il"}, required=True)
    parser.add_argument("--save_every", type=int, default=10)
    parser.add_argument("--update_every", type=int, default=5)
    parser.add_argument("--n_round", type=int, default=2000)
    parser.add_argument("--render", action="store_true")
    parser.add_argument("--map_size", type=int, default=40)
    parser.add_argument("--max_steps", type=int, default=400)
    parser.add_argument("--envs", type=int, default=1, help="envs per round (>1: batched engine in HBM)")
    parser.add_argument("--base_dir", type=str, default=os.getcwd())
    args = parser.parse_args(argv)

    env = magent.GridWorld("battle", map_size=args.map_size)
    env.set_render_dir(os.path.join(args.base_dir, "examples/battle_model", "build/render"))  # train_battle.py:87
    handles = env.get_handles()
    log_dir = os.path.join(args.base_dir, "data/tmp")
    model_dir = os.path.join(args.base_dir, "data/models/{}".format(args.algo))
    # the reference's 80000 replay rows are sized for one env; with E envs keep E times as many
    # (capped at 2M rows = 9.5 GB of views in HBM)
    memory = min(80000 * args.envs, 2000000)
    models = [spawn_ai(args.algo, None, env, handles[0], args.algo + "-me", args.max_steps, memory_size=memory),
              spawn_ai(args.algo, None, env, handles[1], args.algo + "-opponent", args.max_steps, memory_size=memory)]
    play_handle = play
    if args.envs > 1:
        from .battle import BattleBatch
        eng = BattleBatch(args.map_size, args.envs, stream=torch.cuda.current_stream())

        def play_handle(env, n_round, map_size, max_steps, handles, models, print_every, eps=1.0, render=False,
                        train=False):
            return play_batched(eng, n_round, map_size, max_steps, models, print_every, eps, train)
    runner = tools.Runner(None, env, handles, args.map_size, args.max_steps, models, play_handle,
                          render_every=args.save_every if args.render else 0, save_every=args.save_every, tau=0.01,
                          log_name=args.algo, log_dir=log_dir, model_dir=model_dir, train=True)
    for k in range(args.n_round):
        eps = linear_decay(k, [0, int(args.n_round * 0.8), args.n_round], [1, 0.2, 0.1])
        t0 = time.time()
        runner.run(eps, k)
        torch.cuda.synchronize()
        print("[TIME] round {}: {:.2f} s ({} envs)".format(k, time.time() - t0, args.envs))


if __name__ == "__main__":
    main()
