"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

torch-CPU f32 evaluation of the reference networks in eval mode (`src/networks.py`),
driven by a reference-format `state_dict`: the same torch ops the reference runs
(conv2d, batch_norm with running statistics, relu, avg_pool2d, linear), so this is what
`bench.py`'s `cpu_baseline` leg times as the reference's CPU net cost. Numerically it is
the reference (`tests/test_oracle.py` checks it against `tests/golden/nets_full.npz`);
`oracle/nets.py` is the numpy restatement the parity tests use.
"""
import numpy as np
import torch
import torch.nn.functional as F

from .nets import rep_layout

BN_EPS = 1e-5


class TorchNets:
    def __init__(self, sd, mcfg):
        self.mcfg = mcfg
        self.sd = {k: torch.as_tensor(np.asarray(v)) for k, v in sd.items()}

    def _conv(self, x, p, pad):
        return F.conv2d(x, self.sd[p + ".weight"], self.sd[p + ".bias"], padding=pad)

    def _bn(self, x, p):  # networks.py:7-35, eval mode (train_torch.py:164)
        s = self.sd
        return F.batch_norm(x, s[p + ".running_mean"], s[p + ".running_var"], s[p + ".weight"], s[p + ".bias"],
                            False, 0.0, BN_EPS)

    def _res(self, x, p):  # networks.py:19-35
        t = F.relu(self._bn(self._conv(x, p + ".conv1", 1), p + ".bn1"))
        return F.relu(self._bn(self._conv(t, p + ".conv2", 1), p + ".bn2") + x)

    def _block(self, x, p, pad):  # ConvBlock networks.py:7-17
        return F.relu(self._bn(self._conv(x, p + ".conv", pad), p + ".bn"))

    @staticmethod
    def _scale(h):  # networks.py:314-328
        B = h.shape[0]
        f = h.reshape(B, -1)
        mn = f.min(dim=1).values.view(B, 1, 1, 1)
        mx = f.max(dim=1).values.view(B, 1, 1, 1)
        return (h - mn) / (mx - mn + 1e-8)

    def representation(self, x):  # networks.py:94-99, 271-280
        for kind, i in rep_layout(self.mcfg):
            p = f"rep_net.blocks.{i}"
            if kind == "conv":
                x = self._conv(x, p, 1)
            elif kind == "res":
                x = self._res(x, p)
            else:
                x = F.avg_pool2d(x, 2)
        return self._scale(x)

    def prediction(self, h):  # networks.py:225-241
        x = h
        for i in range(self.mcfg["prediction_network"]["num_res_blocks"]):
            x = self._res(x, f"pred_net.res_blocks.{i}")
        s = self.sd
        p = self._block(x, "pred_net.policy_head.0", 1).flatten(1)
        p = F.linear(p, s["pred_net.policy_head.2.weight"], s["pred_net.policy_head.2.bias"])
        v = self._block(x, "pred_net.value_head.0", 0).flatten(1)
        v = F.linear(v, s["pred_net.value_head.2.weight"], s["pred_net.value_head.2.bias"])
        return p, v

    def dynamics(self, h, planes):  # networks.py:151-167, 282-298
        x = self._block(torch.cat([h, planes], 1), "dyn_net.conv_block", 1)
        for i in range(self.mcfg["dynamics_network"]["num_res_blocks"]):
            x = self._res(x, f"dyn_net.res_blocks.{i}")
        s = self.sd
        r = self._block(x, "dyn_net.reward_head.0", 0).flatten(1)
        r = F.linear(r, s["dyn_net.reward_head.2.weight"], s["dyn_net.reward_head.2.bias"])
        return self._scale(x), r


def _decode(logits, smin, smax):  # utils.py:74-81 + :26-28
    sup = torch.linspace(smin, smax, logits.shape[-1])
    x = (torch.softmax(logits, -1) * sup).sum(-1)
    return torch.sign(x) * ((x.abs() + 0.999) ** 2 - 1)


class TorchNetModel:
    """The `model` interface of oracle/mcts.py (root / expand, decoded as mcts.py:95-100,
    194-199) on torch-CPU nets; latents stay torch tensors between calls."""

    def __init__(self, sd, mcfg):
        self.nets = TorchNets(sd, mcfg)
        self.mcfg = mcfg

    def representation(self, x):
        with torch.no_grad():
            return self.nets.representation(torch.as_tensor(x))

    def root(self, h):
        with torch.no_grad():
            p, v = self.nets.prediction(torch.as_tensor(h))
            smin, smax = self.mcfg["supports_min"], self.mcfg["supports_max"]
            return _decode(v, smin, smax).numpy(), torch.softmax(p, 1).numpy()

    def expand(self, parents, actions):
        with torch.no_grad():
            h = torch.as_tensor(parents)
            lh, lw = h.shape[2], h.shape[3]
            planes = F.one_hot(torch.as_tensor(actions), 3).float()[:, :, None, None].expand(-1, -1, lh, lw)
            h2, r = self.nets.dynamics(h, planes)
            p, v = self.nets.prediction(h2)
            smin, smax = self.mcfg["supports_min"], self.mcfg["supports_max"]
            return (h2, _decode(r, smin, smax).numpy(), _decode(v, smin, smax).numpy(),
                    torch.softmax(p, 1).numpy())
