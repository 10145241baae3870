"""Layer-by-layer bf16 vs f32 forward comparison of the learner (first ops of the minibatch)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-breakout_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mzba.config import default_config  # noqa: E402
from mzba.learner import Learner, MinibatchRing  # noqa: E402
from mzba.weights import init_state_dict  # noqa: E402

z = np.load(os.path.join(ROOT, "tests", "golden", "learner_full.npz"))
mcfg = default_config()["model"]
mb = {k.split("/")[-1]: z[k] for k in z.files if k.startswith("s1/in/")}
ring = MinibatchRing(mb)
rec = {}
for dt in ("f32", "bf16"):
    ln = Learner(mcfg, init_state_dict(mcfg, int(z["seed"])), K=int(z["K"]), dtype=dt)
    log = rec.setdefault(dt, [])
    oc, ob = ln._conv, ln._bn

    def conv(c, x, B, H, W, oc=oc, log=log):
        t = oc(c, x, B, H, W)
        log.append(("conv-in", x.float().cpu()))
        log.append(("conv", t.float().cpu()))
        return t

    def bn(c, t, res=None, relu=True, ob=ob, log=log):
        y, s = ob(c, t, res, relu)
        log.append(("bn", y.float().cpu()))
        return y, s
    ln._conv, ln._bn = conv, bn
    ln.train_minibatch(ring, ring.slots())
    torch.cuda.synchronize()
for i, ((n, a), (_, b)) in enumerate(zip(rec["f32"], rec["bf16"])):
    d = (a - b).abs().max().item()
    print(i, n, tuple(a.shape), "max|f32|", round(a.abs().max().item(), 4), "max|diff|", round(d, 5))
    if i > 40:
        break
