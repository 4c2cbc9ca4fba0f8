"""Diagnostic: state after the first fused rollout steps vs the C oracle (positions, hp, rewards)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mean-field-multi-agent-reinforcement-learning_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import numpy as np  # noqa: E402
import battle_driver as bd  # noqa: E402
import common  # noqa: E402
from mfrl_amd.battle import BattleBatch  # noqa: E402

map_size, n_side, E, T = 64, 128, 2, int(sys.argv[1]) if len(sys.argv) > 1 else 3
left, right = bd.block_positions(map_size, n_side)
eng = BattleBatch(map_size, E, stream=torch.cuda.current_stream())
eng.rollout_init([left, right], max_steps=400, eps=0.3, seed=99, stagger=False)
rc = eng.rowcap
envs = []
for e in range(E):
    env, h = common.battle_env(common.ORACLE_LIB, map_size)
    env.reset()
    env.add_agents(h[0], method="custom", pos=left)
    env.add_agents(h[1], method="custom", pos=right)
    envs.append((env, h))
for t in range(T):
    eng.rollout_step(1)
    act = torch.empty(E * 2 * rc, dtype=torch.int32)
    rew = torch.empty(E * 2 * rc, dtype=torch.float32)
    eng.rollout_copy("actions", act)
    eng.rollout_copy("rewards", rew)
    pos = [torch.zeros(E * rc * 2, dtype=torch.int32, device="cuda") for _ in range(2)]
    hp = [torch.zeros(E * rc, dtype=torch.float32, device="cuda") for _ in range(2)]
    num = torch.zeros(E, dtype=torch.int32, device="cuda")
    nums = []
    for g in range(2):
        eng.get(g, 4, pos[g], rc)
        eng.get(g, 5, hp[g], rc)
        eng.get(g, 0, num, rc)
        nums.append(num.cpu().numpy().copy())
    eng.sync()
    for e in range(E):
        env, h = envs[e]
        for g in range(2):
            n = env.get_num(h[g])
            a = act.numpy().reshape(E, 2, rc)[e, g, :n].astype(np.int32)
            env.get_observation(h[g])
            env.set_action(h[g], a)
        env.step()
        rs = [env.get_reward(h[g]) for g in range(2)]
        env.clear_dead()
        for g in range(2):
            r = rs[g]
            gr = rew.numpy().reshape(E, 2, rc)[e, g, :len(r)]
            op = env.get_pos(h[g])
            n = len(op)
            ohp = None
            gp_ = pos[g].cpu().numpy().reshape(E, rc, 2)[e, :n]
            ghp = hp[g].cpu().numpy().reshape(E, rc)[e, :n]
            bad_r = np.nonzero(gr != r)[0]
            bad_p = np.nonzero((gp_ != op).any(1))[0]
            print("t=%d e=%d g=%d n=%d gpu_n=%d  reward mismatches %d %s  pos mismatches %d %s"
                  % (t, e, g, n, nums[g][e], len(bad_r), bad_r[:8].tolist(), len(bad_p), bad_p[:8].tolist()))
            for i in bad_p[:4]:
                print("    agent %d gpu pos %s oracle pos %s action %d" % (i, gp_[i].tolist(), op[i].tolist(),
                      act.numpy().reshape(E, 2, rc)[e, g, i]))
            for i in bad_r[:4]:
                print("    agent %d gpu r %r oracle r %r action %d" % (i, gr[i], r[i], act.numpy().reshape(E, 2, rc)[e, g, i]))
