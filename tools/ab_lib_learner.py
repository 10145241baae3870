"""Learner minibatch time + result hash of ONE build of the C ABI (MZBA_LIB picks it), for same-box A/B of
two builds in alternating processes: bench.py's learner setup (synthetic device ring, bf16 or f32, B = 512,
K = 5), 2 eager minibatches whose gradients and parameters are hashed (sha256 of their bytes: two builds that
must be bit-identical are checked on the same seeded input), then the minibatch as one HIP graph, median of
HIP-event times over 10 replays.
usage (GPU box): MZBA_LIB=muzero-breakout_amd/mzba/libmzba_base.so python tools/ab_lib_learner.py [bf16|f32]
MZBA_WGRAD_FORM=0|1|2 picks the whole-image weight-gradient form of the one build (mzba_conv_wgrad_set_form)."""
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
from mzba.config import default_config  # noqa: E402
from mzba.learner import Learner  # noqa: E402
from mzba.weights import init_state_dict  # noqa: E402


def main():
    dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    mcfg = default_config()["model"]
    dev = torch.device("cuda:0")
    B, K, Lh, cap = 512, 5, mcfg["state_history_length"], 4096
    g = torch.Generator(device=dev).manual_seed(0)

    class Ring:
        pass
    ring = Ring()
    ring.start, ring.max_length, ring.length = 0, cap, cap
    ring._ring = {
        "states": (torch.randint(0, 8, (cap, Lh, 320), device=dev, generator=g) *
                   (torch.rand(cap, Lh, 320, device=dev, generator=g) < 0.3)).to(torch.uint8),
        "past_actions": torch.randint(0, 3, (cap, Lh), device=dev, generator=g),
        "future_actions": torch.randint(0, 3, (cap, K), device=dev, generator=g),
        "rewards": torch.randint(-1, 2, (cap, K), device=dev, generator=g).float(),
        "targets": torch.randn(cap, K, device=dev, generator=g) * 2,
        "counts": torch.randint(0, 51, (cap, K, 3), device=dev, generator=g).float() + 1,
    }
    form = os.environ.get("MZBA_WGRAD_FORM")
    if form is not None:
        from mzba import _lib as L
        L.call("mzba_conv_wgrad_set_form", int(form))
    ln = Learner(mcfg, init_state_dict(mcfg, 0), K=K, dtype=dt, device=dev)
    slots = [torch.randperm(cap, device=dev, generator=g)[:B].to(torch.int32) for _ in range(12)]
    for i in range(2):
        loss = ln.train_minibatch(ring, slots[i])
    torch.cuda.synchronize()
    h = hashlib.sha256()
    h.update(loss.cpu().numpy().tobytes())
    for k, v in sorted(ln.gradients().items()):
        h.update(v.detach().float().cpu().numpy().tobytes())
    for k, v in sorted(ln.state_dict().items()):
        h.update(v.detach().cpu().numpy().tobytes())
    ln.capture(ring, B)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for i in range(10):
        ev[i][0].record()
        ln.train_minibatch(ring, slots[2 + i])
        ev[i][1].record()
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(c) for a, c in ev]))
    print(json.dumps({"lib": os.path.basename(os.environ.get("MZBA_LIB", "libmzba.so")), "dtype": dt, "wgrad_form": form,
                      "minibatch_ms": ms, "sha": h.hexdigest()[:16]}))


if __name__ == "__main__":
    main()
