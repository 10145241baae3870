"""Calibration of the bf16 learner's fused-vs-separate BN statistics check over several seeds
(tests/test_gpu_learner.py test_learner_fused_bn_statistics_track_separate_passes): per seed, the
narrow learner (latent 128) trained one minibatch three ways — bf16 with the separate BN passes,
bf16 with the statistics in the conv epilogues, f32 — and the per-tensor gradient cosines between
them. usage (GPU box): [MZBA_LIB=...] python tools/learner_bn_calib.py [n_seeds]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mzba.config import learner_model_cfg  # noqa: E402
from mzba.learner import Learner  # noqa: E402
from mzba.weights import init_state_dict  # noqa: E402
from test_gpu_learner import _random_ring, _pre_bn_bias  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    mcfg = learner_model_cfg()
    mcfg["latent_channels"] = [128, 128]
    for seed in range(n):
        ring = _random_ring(64, mcfg["state_history_length"], 5, 21 + seed)
        out = {}
        for tag, dt, fuse in (("sep", "bf16", False), ("fused", "bf16", True), ("f32", "f32", False)):
            ln = Learner(mcfg, init_state_dict(mcfg, 4 + seed), K=5, dtype=dt, fuse_bn=fuse, lat_rows="auto")
            out[tag] = (ln.train_minibatch(ring, ring.slots()).cpu(), ln.gradients())
            del ln

        def cos(a, b):
            c = []
            for k, g0 in out[b][1].items():
                if _pre_bn_bias(k) or g0.abs().max() == 0:
                    continue
                c.append(torch.nn.functional.cosine_similarity(g0.flatten().double(), out[a][1][k].flatten().double(),
                                                               dim=0).item())
            return np.array(c)
        r = {"lib": os.environ.get("MZBA_LIB", "libmzba.so"), "seed": seed,
             "loss_rel_fused_sep": float(((out["fused"][0] - out["sep"][0]).abs() / out["sep"][0].abs().clamp_min(1e-6)).max())}
        for a, b in (("fused", "sep"), ("fused", "f32"), ("sep", "f32")):
            c = cos(a, b)
            r[f"{a}~{b}"] = {"min": float(c.min()), "p05": float(np.percentile(c, 5)), "median": float(np.median(c))}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
