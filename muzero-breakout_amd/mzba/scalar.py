"""ScalarTransforms (mirror of utils.py:8-81) and the plugin helpers (utils.py:84-107).

`inverted_softmax_expectation` — the inference-time decode on the hot path — runs in
the HIP kernel `mzba_support_decode` for device tensors (the search itself uses the same
decode fused into the heads kernels). `supports_representation` builds learner targets
(train_torch.py:33-66, out of scope for the acting path) and is plain torch.
"""
import importlib

import torch
import torch.nn as nn

from . import _lib as L


class ScalarTransforms:
    def __init__(self, cfg):
        self.epsilon = 0.001
        self.supports_min = cfg["supports_min"]
        self.supports_max = cfg["supports_max"]
        self.num_supports = cfg["num_supports"]
        dev = cfg.get("device", "cuda")
        self.device = "cuda" if str(dev).startswith("cuda") else dev
        self.supports = torch.linspace(self.supports_min, self.supports_max, self.num_supports).to(self.device)

    def _invertible_transform_normal_to_compact(self, x):
        return torch.sign(x) * (torch.sqrt(torch.abs(x) + 1) - 1 + self.epsilon * x)

    def _invertible_transform_compact_to_normal(self, x):
        return torch.sign(x) * ((torch.abs(x) + (1 - self.epsilon)) ** 2 - 1)

    def supports_representation(self, target_value):
        """utils.py:30-64 (learner targets)."""
        t = self._invertible_transform_normal_to_compact(target_value)
        sup = self.supports.to(t.device)
        lower = (torch.searchsorted(sup, t, right=True) - 1).clamp(0, self.num_supports - 2)
        upper = lower + 1
        ls, us = sup[lower], sup[upper]
        p_low = (us - t) / (us - ls + 1e-10)
        p_high = 1 - p_low
        B, K = target_value.shape
        out = torch.zeros((B, K, self.num_supports), device=t.device)
        out.scatter_(2, lower.unsqueeze(-1), p_low.unsqueeze(-1))
        out.scatter_(2, upper.unsqueeze(-1), p_high.unsqueeze(-1))
        return out

    def _softmax_expectation(self, softmax_distribution):
        return torch.sum(softmax_distribution * self.supports.to(softmax_distribution.device), dim=-1)

    def inverted_softmax_expectation(self, logits):
        """utils.py:74-81 on the HIP path: (..., n) f32 logits -> (...) decoded scalars."""
        L.require_gpu()
        x = logits.to("cuda", torch.float32).contiguous()
        out = L.ops().support_decode(x, float(self.supports_min), float(self.supports_max))
        return out.to(logits.device)


def get_class(module_name, class_name):
    """utils.py:84-96: name-based plugin loading (same error behaviour)."""
    try:
        module = importlib.import_module(module_name)
        return getattr(module, class_name)
    except Exception:
        raise ImportError(f"Could not import module {module_name}")


def torch_activation_map(activation):
    """utils.py:99-107."""
    return {"relu": nn.ReLU, "leaky_relu": nn.LeakyReLU, "silu": nn.SiLU, "gelu": nn.GELU}[activation]
