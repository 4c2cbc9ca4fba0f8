"""ValueNet (algo/base.py:7-279) on PyTorch-ROCm: eval / target Q networks, greedy act, the MF-Q
target on device (HIP kernel mfx_mfq_target), masked-MSE Adam step, soft target update.

Inputs may be numpy arrays (the reference's call sites) or device tensors (the batched engine);
outputs follow the reference: act -> int32 numpy, calc_target_q -> float64, train -> (loss, stats).
"""
import copy

import numpy as np
import torch

from .. import mf, replay
from .nets import QNet


def as_dev(x, dtype=torch.float32):
    if isinstance(x, torch.Tensor):
        return x.to(device="cuda", dtype=dtype)
    return torch.as_tensor(np.asarray(x), dtype=dtype, device="cuda")


def weights_key(net, gen=0):
    """Changes whenever `net`'s weights may have changed: every in-place update of a parameter (optimiser
    steps, copy_, load_state_dict) bumps its version counter; `gen` covers updates torch does not see (a
    replayed HIP graph).  The HIP forwards re-pack their weight blob only when the key moves."""
    return (gen, tuple((p.data_ptr(), p._version) for p in net.parameters()))


class ValueNet:
    graph_train = True          # train() replays the minibatch step as a HIP graph (train_batches)

    def __init__(self, sess, env, handle, name, update_every=5, use_mf=False, learning_rate=1e-4, tau=0.005,
                 gamma=0.95):
        self.env = env
        self.name = name
        self.name_scope = name or "ValueNet"
        self.handle = handle
        self.view_space = tuple(env.get_view_space(handle))
        assert len(self.view_space) == 3
        self.feature_space = tuple(env.get_feature_space(handle))
        self.num_actions = env.get_action_space(handle)[0]
        self.update_every = update_every
        self.use_mf = use_mf
        self.temperature = 0.1
        self.lr = learning_rate
        self.tau = tau
        self.gamma = gamma
        self.eval_net = QNet(self.view_space, self.feature_space, self.num_actions, use_mf).cuda()
        self.target_net = copy.deepcopy(self.eval_net)     # TF initialises both; any start works
        for p in self.target_net.parameters():
            p.requires_grad_(False)
        # capturable: the step count lives on the device, so train_batches can replay the whole
        # minibatch update (sample gather, target, loss, backward, Adam, soft update) as a HIP graph
        self.optimizer = torch.optim.Adam(self.eval_net.parameters(), lr=self.lr, capturable=True)
        self._graph = None
        self._wgen = 0              # bumped after graph replays (they update the weights behind torch's back)
        self._hip_key = None

    @property
    def vars(self):
        """Parameters in a fixed order (eval net, then target net), like the scope's variables."""
        return list(self.eval_net.parameters()) + list(self.target_net.parameters())

    def _prob(self, kwargs, n):
        if not self.use_mf:
            return None
        assert kwargs.get("prob", None) is not None
        return as_dev(kwargs["prob"]).reshape(n, self.num_actions)

    def calc_target_q(self, **kwargs):
        """kwargs: obs, feature, prob (mean field), dones, rewards -> float64 [n] (numpy)."""
        return self.calc_target_q_dev(**kwargs).cpu().numpy()

    @torch.no_grad()
    def calc_target_q_dev(self, **kwargs):
        obs, feat = as_dev(kwargs["obs"]), as_dev(kwargs["feature"])
        prob = self._prob(kwargs, len(obs))
        t_q = self.target_net(obs, feat, prob)
        e_q = self.eval_net(obs, feat, prob)
        return mf.mfq_target(e_q.float().contiguous(), t_q.float().contiguous(), as_dev(kwargs["rewards"]),
                             as_dev(kwargs["dones"], torch.uint8), self.gamma)

    @torch.no_grad()
    def update(self):
        """Soft update: target = tau * eval + (1 - tau) * target."""
        for t, e in zip(self.target_net.parameters(), self.eval_net.parameters()):
            t.mul_(1.0 - self.tau).add_(self.tau * e)

    # ------------------------------------------------------------------ minibatch loop on device
    def train_batches(self, buf, batch_num, use_mean):
        """The reference's train loop (algo/q_learning.py:42-54 DQN, :110-131 MFQ): batch_num times
        sample -> calc_target_q -> train -> update, printing the loss every 50 minibatches.

        The sample indices are drawn up front with the same np.random.choice calls sample() makes,
        and the minibatch step is captured once as a HIP graph (static index tensors, the replay
        rings' fixed storage) and replayed, so a minibatch is one graph launch instead of ~150
        kernel launches and three host syncs.  The first minibatches run eagerly on a side stream
        (the warm-up graph capture needs); the losses are read back once at the end."""
        if batch_num <= 0:
            return
        n, B = buf.nb_entries, buf.batch_size
        idx = np.stack([np.random.choice(n, size=B) for _ in range(batch_num)]).astype(np.int64)
        nxt = (idx + 1) % n
        idx_d = torch.as_tensor(idx, device="cuda")
        nxt_d = torch.as_tensor(nxt, device="cuda")
        stats = torch.zeros((batch_num, 2), dtype=torch.float32, device="cuda")
        if self._graph is None:
            self._s_idx = torch.zeros(B, dtype=torch.int64, device="cuda")
            self._s_nxt = torch.zeros(B, dtype=torch.int64, device="cuda")
            self._s_out = torch.zeros(2, dtype=torch.float32, device="cuda")
        warm = 0 if self._graph is not None else min(3, batch_num)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for i in range(warm):
                self._s_idx.copy_(idx_d[i])
                self._s_nxt.copy_(nxt_d[i])
                self._minibatch(buf, use_mean)
                stats[i].copy_(self._s_out)
        torch.cuda.current_stream().wait_stream(side)
        if warm < batch_num and self._graph is None:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._minibatch(buf, use_mean)
            self._graph = g
        for i in range(warm, batch_num):
            self._s_idx.copy_(idx_d[i])
            self._s_nxt.copy_(nxt_d[i])
            self._graph.replay()
            stats[i].copy_(self._s_out)
        self._wgen += 1
        st = stats.cpu().numpy()
        for i in range(0, batch_num, 50):
            print("[*] LOSS:", float(st[i, 0]), "/ Q:", {"Eval-Q": np.round(float(st[i, 1]), 6)})

    def _minibatch(self, buf, use_mean):
        """One sample + target + masked-MSE Adam step + soft update on the static index tensors."""
        i, j = self._s_idx, self._s_nxt
        # the minibatch rows: one HIP gather (k_rows_copy) per index list, into static tensors the
        # captured graph reuses (allocated by the first, eager call)
        cur = [buf.obs0, buf.feat0, buf.actions, buf.rewards, buf.terminals, buf.masks] + ([buf.prob] if use_mean else [])
        nxt = [buf.obs0, buf.feat0] + ([buf.prob] if use_mean else [])
        if getattr(self, "_mb", None) is None or self._mb[0][0].shape[0] != len(i):
            self._mb = [[torch.empty((len(i),) + tuple(b.data.shape[1:]), dtype=b.data.dtype, device="cuda")
                         for b in bufs] for bufs in (cur, nxt)]
        replay.rows_copy(self._mb[0], [b.data for b in cur], i)
        replay.rows_copy(self._mb[1], [b.data for b in nxt], j)
        obs, feat, acts, rew, done, mask = self._mb[0][:6]
        acts, mask = acts.long(), mask.float()
        obs_n, feat_n = self._mb[1][:2]
        prob = self._mb[0][6] if use_mean else None
        prob_n = self._mb[1][2] if use_mean else None
        with torch.no_grad():
            t_q = self.target_net(obs_n, feat_n, prob_n)
            e_qn = self.eval_net(obs_n, feat_n, prob_n)
            target = mf.mfq_target(e_qn.float().contiguous(), t_q.float().contiguous(), rew, done, self.gamma)
        e_q = self.eval_net(obs, feat, prob)
        e_q_max = e_q.gather(1, acts.reshape(-1, 1)).reshape(-1)
        loss = torch.sum(torch.square(target.float() - e_q_max) * mask) / torch.sum(mask)
        self.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        self.optimizer.step()
        with torch.no_grad():
            t_p = list(self.target_net.parameters())
            e_p = list(self.eval_net.parameters())
            torch._foreach_mul_(t_p, 1.0 - self.tau)
            torch._foreach_add_(t_p, torch._foreach_mul(e_p, self.tau))
            self._s_out[0].copy_(loss.detach())
            self._s_out[1].copy_(e_q_max.detach().mean())

    @torch.no_grad()
    def act_dev(self, **kwargs):
        """Device in, device out: int32 greedy actions (algo/base.py:228-254).  The Battle view runs the
        hand-written HIP forward (mfrl_amd.policy.QNetHIP, csrc/policy_kernels.hip) with the eval net's
        current weights: argmax of e_q, the reference's argmax softmax(e_q / temperature) up to float ties.
        Other view shapes (not in the shipped configs) run the torch module."""
        view, feat = as_dev(kwargs["state"][0]), as_dev(kwargs["state"][1])
        self.temperature = kwargs["eps"]
        prob = self._prob(kwargs, len(view))
        if self.use_mf:
            assert len(prob) == len(view)
        if self.view_space == (13, 13, 7) and self.num_actions <= 32:
            if getattr(self, "_hip", None) is None:
                from ..policy import QNetHIP
                self._hip = QNetHIP(self.view_space, self.feature_space, self.num_actions, self.use_mf)
            key = weights_key(self.eval_net, self._wgen)
            if key != self._hip_key:                     # the weights train() last left, packed once
                self._hip.load(self.eval_net)
                self._hip_key = key
            return self._hip.act(view, feat, prob)
        e_q = self.eval_net(view, feat, prob)
        return torch.argmax(torch.softmax(e_q / self.temperature, dim=1), dim=1).to(torch.int32)

    def act(self, **kwargs):
        return self.act_dev(**kwargs).cpu().numpy().astype(np.int32)

    def train(self, **kwargs):
        """kwargs: state [obs, feature], target_q, prob, acts, masks -> (loss, {'Eval-Q', 'Target-Q'})."""
        obs, feat = as_dev(kwargs["state"][0]), as_dev(kwargs["state"][1])
        prob = self._prob(kwargs, len(obs))
        target = as_dev(kwargs["target_q"])
        mask = as_dev(kwargs["masks"])
        acts = as_dev(kwargs["acts"], torch.int64)
        e_q = self.eval_net(obs, feat, prob)
        e_q_max = e_q.gather(1, acts.reshape(-1, 1)).reshape(-1)
        loss = torch.sum(torch.square(target - e_q_max) * mask) / torch.sum(mask)
        self.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        self.optimizer.step()
        return loss.item(), {"Eval-Q": np.round(e_q_max.mean().item(), 6), "Target-Q": np.round(target.mean().item(), 6)}

    def _save(self, dir_path, prefix, step):
        import os
        os.makedirs(dir_path, exist_ok=True)
        path = os.path.join(dir_path, "{}_{}.pt".format(prefix, step))
        torch.save({"eval": self.eval_net.state_dict(), "target": self.target_net.state_dict()}, path)
        print("[*] Model saved at: {}".format(path))

    def _load(self, dir_path, prefix, step):
        import os
        path = os.path.join(dir_path, "{}_{}.pt".format(prefix, step))
        state = torch.load(path, map_location="cuda", weights_only=True)
        self.eval_net.load_state_dict(state["eval"])
        self.target_net.load_state_dict(state["target"])
        print("[*] Loaded model from {}".format(path))
