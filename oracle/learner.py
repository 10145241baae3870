"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

Restatement of one learner minibatch of the reference as a functional
torch-CPU f32 program over a reference-format state dict (the checker for the HIP learner,
a floating-point path, so torch f32 is the reference arithmetic):

* input  — `_prepare_minibatch` + `_encode_actions` (train_torch.py:437-470, 279-293): the 32
  window frames, then the 32 past actions as a/3 planes;
* forward — `_k_step_rollout` (train_torch.py:487-528): representation + min-max scale, then K
  times prediction(h_k) and dynamics(h_k, one-hot a_k) (`_encode_action_dynamics` :295-311),
  every BatchNorm in train mode (batch statistics, running-stat update, networks.py:344-350);
* loss   — `loss_fn` (train_torch.py:33-66): three KL(batchmean) terms against
  `supports_representation` targets (utils.py:30-64) and normalised visit counts, times 1/K;
* update — `torch.optim.Adam(lr, weight_decay=1e-4)` (networks.py:268), the single-tensor
  algorithm: g += wd p; m = lerp(m, g, 1 - b1); v = b2 v + (1 - b2) g^2;
  p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps).

Pinned against the reference's own training step in tests/golden/learner_*.npz
(tests/golden/make_golden.py make_learner).
"""
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

BN_EPS, BN_MOMENTUM = 1e-5, 0.1
ADAM_BETAS, ADAM_EPS, WEIGHT_DECAY = (0.9, 0.999), 1e-8, 1e-4


def rep_layout(mcfg):
    n0, n1, n2 = mcfg["representation_network"]["num_res_blocks"]
    seq, i = [("conv", 0)], 1
    for n, tail in ((n0, "conv"), (n1, "pool"), (n2, "pool")):
        for _ in range(n):
            seq.append(("res", i)); i += 1
        seq.append((tail, i)); i += 1
    return seq


def supports_representation(x, smin, smax, n, eps=0.001):
    """utils.py:30-64: compact transform, two-hot over linspace(smin, smax, n)."""
    sup = torch.linspace(smin, smax, n, dtype=x.dtype)
    t = torch.sign(x) * (torch.sqrt(torch.abs(x) + 1) - 1 + eps * x)
    lo = (torch.searchsorted(sup, t, right=True) - 1).clamp(0, n - 2)
    hi = lo + 1
    pl = (sup[hi] - t) / (sup[hi] - sup[lo] + 1e-10)
    out = torch.zeros(*x.shape, n, dtype=x.dtype)
    out.scatter_(-1, lo.unsqueeze(-1), pl.unsqueeze(-1))
    out.scatter_(-1, hi.unsqueeze(-1), (1 - pl).unsqueeze(-1))
    return out


def kl_batchmean(logits, target):
    logp = F.log_softmax(logits.reshape(-1, logits.shape[-1]), dim=-1)
    t = target.reshape(-1, logits.shape[-1])
    return F.kl_div(logp, t, reduction="batchmean")


class LearnerOracle:
    """Parameters, BN running stats and Adam state of the three nets; `step(minibatch)`."""

    def __init__(self, mcfg, state_dict, K=5, lr=None, dtype=torch.float32):
        self.m, self.K, self.dtype = mcfg, K, dtype
        self.lr = mcfg["learning_rate"] if lr is None else lr
        self.p, self.buf = OrderedDict(), OrderedDict()
        for k, v in state_dict.items():
            t = torch.tensor(np.asarray(v))
            if k.endswith(("running_mean", "running_var")):
                self.buf[k] = t.clone().to(dtype)
            elif k.endswith("num_batches_tracked"):
                self.buf[k] = t.clone()
            else:
                self.p[k] = t.clone().to(dtype).requires_grad_(True)
        self.adam = {k: [0, torch.zeros_like(v), torch.zeros_like(v)] for k, v in self.p.items()}

    # -- modules -----------------------------------------------------------------------------
    def _conv(self, x, pre, pad):
        return F.conv2d(x, self.p[pre + ".weight"], self.p[pre + ".bias"], padding=pad)

    def _bn(self, x, pre):
        self.buf[pre + ".num_batches_tracked"] += 1
        return F.batch_norm(x, self.buf[pre + ".running_mean"], self.buf[pre + ".running_var"], self.p[pre + ".weight"],
                            self.p[pre + ".bias"], training=True, momentum=BN_MOMENTUM, eps=BN_EPS)

    def _res(self, x, pre):
        y = F.relu(self._bn(self._conv(x, pre + ".conv1", 1), pre + ".bn1"))
        return F.relu(self._bn(self._conv(y, pre + ".conv2", 1), pre + ".bn2") + x)

    def _block(self, x, pre, pad):  # ConvBlock (networks.py:7-17)
        return F.relu(self._bn(self._conv(x, pre + ".conv", pad), pre + ".bn"))

    def _linear(self, x, pre):
        return F.linear(x.flatten(1), self.p[pre + ".weight"], self.p[pre + ".bias"])

    force_index = None  # optional list of (B, 2) NCHW-flat (argmin, argmax) per _scale call

    def _scale(self, h):
        f = h.view(h.shape[0], -1)
        if self.force_index is not None:
            # the min / max taken at given positions: the same values up to rounding near-ties, and
            # the gradient routed to those positions (torch.min/max(dim) route to their index)
            idx = torch.as_tensor(np.asarray(self.force_index[self._nscale]), dtype=torch.int64)
            self._nscale += 1
            mn = f.gather(1, idx[:, :1]).view(-1, 1, 1, 1)
            mx = f.gather(1, idx[:, 1:2]).view(-1, 1, 1, 1)
        else:
            mn = f.min(dim=1, keepdim=True)[0].view(-1, 1, 1, 1)
            mx = f.max(dim=1, keepdim=True)[0].view(-1, 1, 1, 1)
        return (h - mn) / (mx - mn + 1e-8)

    def representation(self, x):
        for kind, i in rep_layout(self.m):
            pre = f"rep_net.blocks.{i}"
            if kind == "conv":
                x = self._conv(x, pre, 1)
            elif kind == "res":
                x = self._res(x, pre)
            else:
                x = F.avg_pool2d(x, 2, 2)
        return self._scale(x)

    def prediction(self, h):
        for i in range(self.m["prediction_network"]["num_res_blocks"]):
            h = self._res(h, f"pred_net.res_blocks.{i}")
        pol = self._linear(self._block(h, "pred_net.policy_head.0", 1), "pred_net.policy_head.2")
        val = self._linear(self._block(h, "pred_net.value_head.0", 0), "pred_net.value_head.2")
        return pol, val

    def dynamics(self, h, a):
        B, _, H, W = h.shape
        planes = F.one_hot(a, 3).to(self.dtype).view(B, 3, 1, 1).expand(-1, -1, H, W)
        x = self._block(torch.cat([h, planes], 1), "dyn_net.conv_block", 1)
        for i in range(self.m["dynamics_network"]["num_res_blocks"]):
            x = self._res(x, f"dyn_net.res_blocks.{i}")
        r = self._linear(self._block(x, "dyn_net.reward_head.0", 0), "dyn_net.reward_head.2")
        return self._scale(x), r

    # -- one minibatch --------------------------------------------------------------------------
    def forward_loss(self, mb):
        self._nscale = 0
        L = self.m["state_history_length"]
        dt = self.dtype
        states = torch.from_numpy(np.asarray(mb["states"], np.float32)).to(dt)
        B = states.shape[0]
        acts = torch.from_numpy(np.asarray(mb["past_actions"], np.int64))
        planes = (acts.to(dt) / 3)[:, :, None, None].expand(-1, -1, 16, 20)
        x = torch.cat([states.view(B, L, 16, 20), planes], 1)
        h = self.representation(x)
        fut = torch.from_numpy(np.asarray(mb["future_actions"], np.int64))
        pols, vals, rews = [], [], []
        for k in range(self.K):
            p, v = self.prediction(h)
            pols.append(p); vals.append(v)
            h, r = self.dynamics(h, fut[:, k])
            rews.append(r)
        pr, pv, pp = torch.stack(rews, 1), torch.stack(vals, 1), torch.stack(pols, 1)
        s = (self.m["supports_min"], self.m["supports_max"], self.m["num_supports"])
        rl = kl_batchmean(pr, supports_representation(torch.from_numpy(np.asarray(mb["rewards"], np.float32)).to(dt), *s))
        vl = kl_batchmean(pv, supports_representation(torch.from_numpy(np.asarray(mb["targets"], np.float32)).to(dt), *s))
        c = torch.from_numpy(np.asarray(mb["counts"], np.float32)).to(dt)
        pl = kl_batchmean(pp, c / c.sum(dim=-1, keepdim=True))
        loss = (1 / self.K) * (rl + vl + pl)
        return loss, (rl, vl, pl), (pr, pv, pp)

    def gradients(self, mb):
        """loss.backward() only (no update): (loss parts, logits, grads)."""
        for v in self.p.values():
            v.grad = None
        loss, parts, logits = self.forward_loss(mb)
        loss.backward()
        return parts, [x.detach() for x in logits], {k: v.grad.detach().clone() for k, v in self.p.items()}

    def step(self, mb):
        for v in self.p.values():
            v.grad = None
        loss, parts, logits = self.forward_loss(mb)
        loss.backward()
        grads = {k: v.grad.detach().clone() for k, v in self.p.items()}
        b1, b2 = ADAM_BETAS
        with torch.no_grad():
            for k, prm in self.p.items():
                st = self.adam[k]
                st[0] += 1
                t = st[0]
                g = prm.grad.add(prm, alpha=WEIGHT_DECAY)
                st[1].lerp_(g, 1 - b1)
                st[2].mul_(b2).addcmul_(g, g, value=1 - b2)
                step_size = self.lr / (1 - b1 ** t)
                denom = (st[2].sqrt() / ((1 - b2 ** t) ** 0.5)).add_(ADAM_EPS)
                prm.addcdiv_(st[1], denom, value=-step_size)
        return dict(loss=float(loss.detach()), parts=[float(x.detach()) for x in parts], logits=[x.detach() for x in logits],
                    grads=grads)

    def state_dict(self):
        out = OrderedDict()
        for k in list(self.p) + list(self.buf):
            out[k] = (self.p[k] if k in self.p else self.buf[k]).detach().clone()
        return out
