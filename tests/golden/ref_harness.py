"""Import shim for the read-only reference at /root/reference (fixture generation ONLY).

Used by tests/golden/make_golden.py in the build container. Never imported by the
product, by `-m gpu` tests, by smoke() or by bench.py (the reference does not exist
on the GPU box). Nothing in the reference is edited: the shims live here.

Shims:
  1. sys.path + dont_write_bytecode (the mount is read-only)
  2. stub `torchvision`, `torchvision.transforms` (unused import, networks.py:5)
  3. stub `torch.utils.tensorboard.SummaryWriter` (train_torch.py:10)
  4. remap device "cuda" -> "cpu" (networks.py:249/278, mcts.py:190)
"""
import sys
import types

REF = "/root/reference"


def install():
    if getattr(install, "_done", False):
        return
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")
    tv.transforms = tvt
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.transforms", tvt)
    import torch
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:  # noqa: D401 - stub
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, name):
            return lambda *a, **k: None

    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb

    def _fix(dev):
        if isinstance(dev, str) and dev.startswith("cuda"):
            return "cpu"
        if isinstance(dev, torch.device) and dev.type == "cuda":
            return torch.device("cpu")
        return dev

    _tto = torch.Tensor.to

    def tensor_to(self, *args, **kwargs):
        args = tuple(_fix(a) for a in args)
        if "device" in kwargs:
            kwargs["device"] = _fix(kwargs["device"])
        return _tto(self, *args, **kwargs)

    torch.Tensor.to = tensor_to
    _mto = torch.nn.Module.to

    def module_to(self, *args, **kwargs):
        args = tuple(_fix(a) for a in args)
        if "device" in kwargs:
            kwargs["device"] = _fix(kwargs["device"])
        return _mto(self, *args, **kwargs)

    torch.nn.Module.to = module_to
    install._done = True


def load_config():
    import yaml
    with open(f"{REF}/config.yaml") as f:
        cfg = yaml.safe_load(f)["parameters"]
    cfg["model"]["device"] = "cpu"
    return cfg
