"""How far apart can two training-loss gradients of this network be when the arithmetic differs
slightly? f32 learner at p vs f32 learner at p * (1 + eps n) for eps = 1e-6, 1e-4, 1e-3, and the
bf16 learner vs f32 — per-tensor gradient cosines (min / median), full config, B = 256."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-breakout_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mzba.config import default_config, learner_model_cfg  # noqa: E402
from mzba.learner import Learner  # noqa: E402
from mzba.weights import init_state_dict  # noqa: E402
from test_gpu_learner import _random_ring, _pre_bn_bias  # noqa: E402

for tag, mcfg in (("small", learner_model_cfg()), ("full", default_config()["model"])):
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    ring = _random_ring(B, mcfg["state_history_length"], 5, 11)
    sd = init_state_dict(mcfg, 5)

    def grads(sd, dt="f32"):
        ln = Learner(mcfg, sd, K=5, dtype=dt)
        loss = ln.train_minibatch(ring, ring.slots()).cpu().numpy()
        return loss, ln.gradients()
    l0, g0 = grads(sd)
    rng = np.random.default_rng(1)

    def cmp(name, l1, g1):
        cos = []
        for k, g in g0.items():
            if g.numel() < 1000 or _pre_bn_bias(k):
                continue
            a, b = g.reshape(-1).double(), g1[k].reshape(-1).double()
            cos.append(float(a @ b / (a.norm() * b.norm() + 1e-30)))
        cos = np.array(cos)
        print(f"{tag} B={B} {name:10s} loss {l1[0]:.5f} vs {l0[0]:.5f}  cos min {cos.min():.4f} median {np.median(cos):.4f}",
              flush=True)
    for eps in (1e-6, 1e-4, 1e-3):
        sdp = {k: (np.asarray(v) * (1 + eps * rng.standard_normal(np.shape(v)))).astype(np.float32)
               if np.asarray(v).dtype == np.float32 and not k.endswith(("running_mean", "running_var")) else v
               for k, v in sd.items()}
        cmp(f"eps={eps:g}", *grads(sdp))
    cmp("bf16", *grads(sd, "bf16"))
