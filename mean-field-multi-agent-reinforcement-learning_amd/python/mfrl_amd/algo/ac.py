"""ActorCritic and MFAC of algo/ac.py:8-361 on PyTorch-ROCm.

act samples the clipped softmax policy (tf.multinomial of its log) on the hand-written HIP forward
(mfrl_amd.policy.ACNetHIP, csrc/acnet_kernels.hip: the policy and a counter-hash draw, its weights re-packed
only when training changed them); train builds one batch from the
episode buffer, bootstraps every agent's sequence from the value of its last row, and runs the
discounted-return recursion keep = keep * gamma + r on the device (HIP kernel mfx_mfac_returns,
algo/ac.py:305-320), then one Adam step on pg + value_coef * vf + ent_coef * neg_entropy.
"""
import os
import zlib

import numpy as np
import torch

from .. import mf
from . import tools
from .base import as_dev, weights_key
from .nets import ACNet


class ActorCritic:
    _prefix = "ac"
    _use_mf = False

    def __init__(self, sess, name, handle, env, value_coef=0.1, ent_coef=0.08, gamma=0.95, batch_size=64,
                 learning_rate=1e-4):
        self.env = env
        self.name = name
        self.name_scope = name
        self.view_space = tuple(env.get_view_space(handle))
        self.feature_space = tuple(env.get_feature_space(handle))
        self.num_actions = env.get_action_space(handle)[0]
        self.gamma = gamma
        self.reward_decay = gamma
        self.batch_size = batch_size
        self.learning_rate = learning_rate
        self.value_coef = value_coef
        self.ent_coef = ent_coef
        self.replay_buffer = tools.EpisodesBuffer(use_mean=self._use_mf)
        self.net = ACNet(self.view_space, self.feature_space, self.num_actions, use_mf=self._use_mf).cuda()
        self.optimizer = torch.optim.Adam(self.net.parameters(), lr=self.learning_rate)
        self._hip = None
        self._hip_key = None
        self._draws = 0             # act() calls: the step counter of the device draw
        # the draw's seed: the run's torch seed mixed with the model name, so runs seeded alike draw alike and
        # differently seeded runs differ, as tf.multinomial under TF's seed would; np.random is left
        # alone -- the reference consumes it in the replay buffers, and seeded runs must draw the same indices
        self.seed = zlib.crc32(("%s/%s/%d" % (self._prefix, name, torch.initial_seed())).encode())

    @property
    def vars(self):
        return list(self.net.parameters())

    def flush_buffer(self, **kwargs):
        self.replay_buffer.push(**kwargs)

    @torch.no_grad()
    def act_dev(self, **kwargs):
        """Device in, device out: int32 actions drawn from the clipped softmax policy (algo/ac.py:43-46,
        tf.multinomial(log(policy))) by the HIP forward k_acnet; the draw's uniforms are a counter hash of
        (self.seed, the act() count, the row) instead of TensorFlow's stream."""
        view, feat = as_dev(kwargs["state"][0]), as_dev(kwargs["state"][1])
        if self._hip_ok():
            self._draws += 1
            return self._hip_net().act(view, feat, seed=self.seed, step=self._draws)
        policy, _ = self.net(view, feat, need_value=False)
        return torch.multinomial(policy, 1).reshape(-1).to(torch.int32)

    def _hip_net(self):
        """The HIP forward with the network's current weights (re-packed only after they changed)."""
        if self._hip is None:
            from ..policy import ACNetHIP
            self._hip = ACNetHIP(self.view_space, self.feature_space, self.num_actions, self._use_mf)
        key = weights_key(self.net)
        if key != self._hip_key:
            self._hip.load(self.net)
            self._hip_key = key
        return self._hip

    def _hip_ok(self):
        return 2 <= self.num_actions <= 32 and int(np.prod(self.view_space)) <= 4096 and self.feature_space[0] <= 256

    def act(self, **kwargs):
        return self.act_dev(**kwargs).cpu().numpy().astype(np.int32)

    def losses(self, view, feature, action, reward, prob=None):
        policy, value = self.net(view, feature, prob)
        action_mask = torch.nn.functional.one_hot(action.long(), self.num_actions).float()
        advantage = (reward - value).detach()
        log_policy = torch.log(policy + 1e-6)
        log_prob = torch.sum(log_policy * action_mask, dim=1)
        pg_loss = -torch.mean(advantage * log_prob)
        vf_loss = self.value_coef * torch.mean(torch.square(reward - value))
        neg_entropy = self.ent_coef * torch.mean(torch.sum(policy * log_policy, dim=1))
        return pg_loss, vf_loss, neg_entropy, value

    def train(self):
        got = self.replay_buffer.batch()
        self.replay_buffer = tools.EpisodesBuffer(use_mean=self._use_mf)
        if got is None:
            return
        rows, counts = got
        view, feature, action = rows["obs"], rows["feat"], rows["act"]
        reward = rows["rew"].clone()
        prob = rows.get("prob")
        last = torch.cumsum(counts, 0) - 1
        with torch.no_grad():                     # value of every agent's last row (the bootstrap), on k_acnet
            if self._hip_ok():
                _, keep, _ = self._hip_net().forward(view[last], feature[last], prob[last] if prob is not None else None,
                                                     want_policy=False, want_value=True, want_act=False)
            else:
                _, keep = self.net(view[last], feature[last], prob[last] if prob is not None else None)
        offsets = torch.zeros(len(counts) + 1, dtype=torch.int64, device="cuda")
        offsets[1:] = torch.cumsum(counts, 0)
        mf.mfac_returns(reward, offsets, keep.float().contiguous(), self.gamma)
        pg_loss, vf_loss, ent_loss, state_value = self.losses(view, feature, action, reward, prob)
        total = pg_loss + vf_loss + ent_loss
        self.optimizer.zero_grad(set_to_none=True)
        total.backward()
        self.optimizer.step()
        print("[*] PG_LOSS:", np.round(pg_loss.item(), 6), "/ VF_LOSS:", np.round(vf_loss.item(), 6),
              "/ ENT_LOSS:", np.round(ent_loss.item(), 6), "/ VALUE:", state_value.mean().item())

    def save(self, dir_path, step=0):
        os.makedirs(dir_path, exist_ok=True)
        path = os.path.join(dir_path, "{}_{}.pt".format(self._prefix, step))
        torch.save(self.net.state_dict(), path)
        print("[*] Model saved at: {}".format(path))

    def load(self, dir_path, step=0):
        path = os.path.join(dir_path, "{}_{}.pt".format(self._prefix, step))
        self.net.load_state_dict(torch.load(path, map_location="cuda", weights_only=True))
        print("[*] Loaded model from {}".format(path))


class MFAC(ActorCritic):
    _prefix = "mfac"
    _use_mf = True
