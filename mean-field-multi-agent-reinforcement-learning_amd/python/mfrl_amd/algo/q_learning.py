"""DQN (IL) and MFQ of algo/q_learning.py:10-143 on the device ValueNet and MemoryGroup."""
from . import base
from . import tools


class DQN(base.ValueNet):
    def __init__(self, sess, name, handle, env, sub_len, memory_size=2 ** 10, batch_size=64, update_every=5):
        super().__init__(sess, env, handle, name, update_every=update_every)
        self.replay_buffer = tools.MemoryGroup(self.view_space, self.feature_space, self.num_actions, memory_size,
                                               batch_size, sub_len)

    def flush_buffer(self, **kwargs):
        self.replay_buffer.push(**kwargs)

    def train(self):
        self.replay_buffer.tight()
        batch_num = self.replay_buffer.get_batch_num()
        if self.graph_train:
            return self.train_batches(self.replay_buffer, batch_num, use_mean=False)
        for i in range(batch_num):
            obs, feats, obs_next, feat_next, dones, rewards, actions, masks = self.replay_buffer.sample()
            target_q = self.calc_target_q_dev(obs=obs_next, feature=feat_next, rewards=rewards, dones=dones)
            loss, q = super().train(state=[obs, feats], target_q=target_q, acts=actions, masks=masks)
            self.update()
            if i % 50 == 0:
                print("[*] LOSS:", loss, "/ Q:", q)

    def save(self, dir_path, step=0):
        self._save(dir_path, "dqn", step)

    def load(self, dir_path, step=0):
        self._load(dir_path, "dqn", step)


class MFQ(base.ValueNet):
    def __init__(self, sess, name, handle, env, sub_len, eps=1.0, update_every=5, memory_size=2 ** 10, batch_size=64):
        super().__init__(sess, env, handle, name, use_mf=True, update_every=update_every)
        self.train_ct = 0
        self.replay_buffer = tools.MemoryGroup(self.view_space, self.feature_space, self.num_actions, memory_size,
                                               batch_size, sub_len, use_mean=True)
        self.update_every = update_every

    def flush_buffer(self, **kwargs):
        self.replay_buffer.push(**kwargs)

    def train(self):
        self.replay_buffer.tight()
        batch_num = self.replay_buffer.get_batch_num()
        if self.graph_train:
            return self.train_batches(self.replay_buffer, batch_num, use_mean=True)
        for i in range(batch_num):
            obs, feat, acts, act_prob, obs_next, feat_next, act_prob_next, rewards, dones, masks = \
                self.replay_buffer.sample()
            target_q = self.calc_target_q_dev(obs=obs_next, feature=feat_next, rewards=rewards, dones=dones,
                                              prob=act_prob_next)
            loss, q = super().train(state=[obs, feat], target_q=target_q, prob=act_prob, acts=acts, masks=masks)
            self.update()
            if i % 50 == 0:
                print("[*] LOSS:", loss, "/ Q:", q)

    def save(self, dir_path, step=0):
        self._save(dir_path, "mfq", step)

    def load(self, dir_path, step=0):
        self._load(dir_path, "mfq", step)
