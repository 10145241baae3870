"""Same-process check of the fused BN finaliser (Learner fuse_fin): counter words used per minibatch, eager and
graph-replayed minibatch times with fuse_fin on / off (bf16, B = 512, K = 5, full nets), alternating."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
from mzba.config import default_config  # noqa: E402
from mzba.learner import Learner  # noqa: E402
from mzba.weights import init_state_dict  # noqa: E402


def ring_of(dev, cap, Lh, K, g):
    class Ring:
        pass
    r = Ring()
    r.start, r.max_length, r.length = 0, cap, cap
    r._ring = {
        "states": (torch.randint(0, 8, (cap, Lh, 320), device=dev, generator=g) *
                   (torch.rand(cap, Lh, 320, device=dev, generator=g) < 0.3)).to(torch.uint8),
        "past_actions": torch.randint(0, 3, (cap, Lh), device=dev, generator=g),
        "future_actions": torch.randint(0, 3, (cap, K), device=dev, generator=g),
        "rewards": torch.randint(-1, 2, (cap, K), device=dev, generator=g).float(),
        "targets": torch.randn(cap, K, device=dev, generator=g) * 2,
        "counts": torch.randint(0, 51, (cap, K, 3), device=dev, generator=g).float() + 1,
    }
    return r


def timed(fn, n):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[n // 2]


def main():
    mcfg = default_config()["model"]
    dev = torch.device("cuda:0")
    B, K, cap = 512, 5, 4096
    g = torch.Generator(device=dev).manual_seed(0)
    ring = ring_of(dev, cap, mcfg["state_history_length"], K, g)
    slots = torch.randperm(cap, device=dev, generator=g)[:B].to(torch.int32)
    lns = {f: Learner(mcfg, init_state_dict(mcfg, 0), K=K, dtype="bf16", device=dev, fuse_fin=f) for f in (False, True)}
    for f, ln in lns.items():
        ln.train_minibatch(ring, slots)
    torch.cuda.synchronize()
    eager = {f: [] for f in lns}
    for _ in range(3):
        for f, ln in lns.items():
            eager[f].append(timed(lambda: ln._minibatch(ring, slots), 3))
    for f, ln in lns.items():
        ln.capture(ring, B)
    graph = {f: [] for f in lns}
    for _ in range(3):
        for f, ln in lns.items():
            graph[f].append(timed(lambda: ln.train_minibatch(ring, slots), 5))
    for f, ln in lns.items():
        print(json.dumps({"fuse_fin": f, "ctr_words_used": ln._ctr_i, "eager_ms": eager[f], "graph_ms": graph[f]}))


if __name__ == "__main__":
    main()
