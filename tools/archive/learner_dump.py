"""Dump the HIP learner's gradients, logits and scale routing for the learner fixtures (small step
1, teacher-forced small step 2, full step 1) to gpurun_out/learner_dump.npz for offline analysis."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-breakout_amd")]
import numpy as np  # noqa: E402
from mzba.config import default_config, learner_model_cfg  # noqa: E402
from mzba.learner import Learner, MinibatchRing  # noqa: E402
from mzba.weights import init_state_dict  # noqa: E402

out = {}


def mb_of(z, s):
    return {k.split("/")[-1]: z[k] for k in z.files if k.startswith(f"s{s}/in/")}


def dump(ln, tag, grads=True):
    for i, a in enumerate(ln.scale_indices()):
        out[f"{tag}/idx{i}"] = a
    for i, t in enumerate(ln.last_logits):
        out[f"{tag}/logits{i}"] = t.cpu().numpy()
    if grads:
        for k, g in ln.gradients().items():
            out[f"{tag}/grad/{k}"] = g.numpy()


z = np.load(os.path.join(ROOT, "tests", "golden", "learner_small.npz"))
mcfg = learner_model_cfg()
ln = Learner(mcfg, init_state_dict(mcfg, int(z["seed"])), K=int(z["K"]))
ring = MinibatchRing(mb_of(z, 1))
ln.train_minibatch(ring, ring.slots())
dump(ln, "small1")
ln.load_state_dict({k[len("s1/param/"):]: z[k] for k in z.files if k.startswith("s1/param/")})
ring = MinibatchRing(mb_of(z, 2))
ln.train_minibatch(ring, ring.slots())
dump(ln, "small2")
z = np.load(os.path.join(ROOT, "tests", "golden", "learner_full.npz"))
mcfg = default_config()["model"]
ln = Learner(mcfg, init_state_dict(mcfg, int(z["seed"])), K=int(z["K"]))
ring = MinibatchRing(mb_of(z, 1))
ln.train_minibatch(ring, ring.slots())
dump(ln, "full1", grads=False)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "learner_dump.npz"), **out)
print("dumped", len(out))
