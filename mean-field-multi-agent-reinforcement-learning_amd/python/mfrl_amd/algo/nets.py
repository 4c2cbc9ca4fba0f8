"""PyTorch networks of the reference's TF1 models (examples/battle_model/algo), layer for layer.

* QNet      = ValueNet._construct_net (algo/base.py:128-188): Conv1/Conv2 (32 filters, 3x3, valid)
              -> Dense-Obs 256; Dense-Emb 32 on the features; with mean field Prob-Emb 64 ->
              Dense-Act-Prob 32; Dense2 128 -> Dense-Out 64 -> Q-Value (linear), ReLU elsewhere.
* ACNet     = ActorCritic._create_network (algo/ac.py:53-98): dense 256 on the flat view and on the
              features -> dense 512 -> policy softmax(dense(x / 0.1)) clipped to [1e-10, 1 - 1e-10],
              value dense(x -> 1).
* MFACNet   = MFAC._create_network (algo/ac.py:219-276): the AC policy branch; the value head sees
              the AC concat layer plus the mean action (64 -> 32) through dense 256.

Views arrive NHWC (the engine's [n, 13, 13, 7] layout); flattening keeps TF's NHWC order so a
layer's weight matrix has the reference's row order.  Initialisation is TF1's default: Glorot
uniform kernels, zero biases.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


def _tf_init(m):
    if isinstance(m, (nn.Linear, nn.Conv2d)):
        nn.init.xavier_uniform_(m.weight)
        nn.init.zeros_(m.bias)


class QNet(nn.Module):
    def __init__(self, view_space, feature_space, num_actions, use_mf=False):
        super().__init__()
        h, w, c = view_space
        self.use_mf = use_mf
        self.conv1 = nn.Conv2d(c, 32, 3)
        self.conv2 = nn.Conv2d(32, 32, 3)
        self.dense_obs = nn.Linear(32 * (h - 4) * (w - 4), 256)
        self.dense_emb = nn.Linear(feature_space[0], 32)
        width = 256 + 32
        if use_mf:
            self.prob_emb = nn.Linear(num_actions, 64)
            self.dense_act_prob = nn.Linear(64, 32)
            width += 32
        self.dense2 = nn.Linear(width, 128)
        self.dense_out = nn.Linear(128, 64)
        self.q_value = nn.Linear(64, num_actions)
        self.apply(_tf_init)

    def forward(self, view, feature, prob=None):
        x = F.relu(self.conv1(view.permute(0, 3, 1, 2)))
        x = F.relu(self.conv2(x))
        x = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)          # TF NHWC flatten order
        h = torch.cat([F.relu(self.dense_obs(x)), F.relu(self.dense_emb(feature))], dim=1)
        if self.use_mf:
            p = F.relu(self.dense_act_prob(F.relu(self.prob_emb(prob))))
            h = torch.cat([h, p], dim=1)
        return self.q_value(F.relu(self.dense_out(F.relu(self.dense2(h)))))


class ACNet(nn.Module):
    def __init__(self, view_space, feature_space, num_actions, use_mf=False, hidden=256):
        super().__init__()
        flat = 1
        for d in view_space:
            flat *= d
        self.use_mf = use_mf
        self.h_view = nn.Linear(flat, hidden)
        self.h_emb = nn.Linear(feature_space[0], hidden)
        self.dense = nn.Linear(2 * hidden, 2 * hidden)
        self.policy = nn.Linear(2 * hidden, num_actions)
        if use_mf:
            self.emb_prob = nn.Linear(num_actions, 64)
            self.dense_prob = nn.Linear(64, 32)
            self.value_dense = nn.Linear(2 * hidden + 32, hidden)
            self.value = nn.Linear(hidden, 1)
        else:
            self.value = nn.Linear(2 * hidden, 1)
        self.apply(_tf_init)

    def forward(self, view, feature, prob=None, need_value=True):
        """-> (policy [n, A] clipped softmax, value [n] or None)."""
        concat = torch.cat([F.relu(self.h_view(view.reshape(view.shape[0], -1))), F.relu(self.h_emb(feature))], dim=1)
        dense = F.relu(self.dense(concat))
        policy = torch.clamp(torch.softmax(self.policy(dense / 0.1), dim=1), 1e-10, 1 - 1e-10)
        if not need_value:
            return policy, None
        if self.use_mf:
            p = F.relu(self.dense_prob(F.relu(self.emb_prob(prob))))
            value = self.value(F.relu(self.value_dense(torch.cat([concat, p], dim=1))))
        else:
            value = self.value(dense)
        return policy, value.reshape(-1)
