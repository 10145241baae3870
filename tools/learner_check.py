"""Learner parity diagnostics (prints every tensor, no early stop): the HIP learner's step-1
gradients on tests/golden/learner_small.npz against the f64 oracle (with the reference's own
f32 error beside them), on learner_full.npz against the reference's per-tensor |grad| sums, and
the bf16 path's gradient cosines against the f32 path.
usage: python tools/learner_check.py [small|full|bf16]...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-breakout_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mzba.config import default_config, learner_model_cfg  # noqa: E402
from mzba.learner import Learner, MinibatchRing  # noqa: E402
from mzba.weights import init_state_dict  # noqa: E402


def mb_of(z, s):
    return {k.split("/")[-1]: z[k] for k in z.files if k.startswith(f"s{s}/in/")}


which = sys.argv[1:] or ["small", "full", "bf16"]
def report(ln, mcfg, start, mb, K, tag):
    from oracle.learner import LearnerOracle
    torch.set_num_threads(16)
    o = LearnerOracle(mcfg, start, K=K, dtype=torch.float64)
    o.force_index = ln.scale_indices()
    _, lg64, g64 = o.gradients(mb)
    for got, key, a in zip(ln.last_logits, ("pr", "pv", "pp"), lg64):
        e = np.abs(got.cpu().numpy().transpose(1, 0, 2) - a.numpy()).max()
        print(f"  {tag} logits {key}: ours-f64 {e:.3e}")
    for k, g in ln.gradients().items():
        t = g64[k].numpy()
        e = np.abs(g.numpy() - t).max()
        print(f"  {tag} {k:45s} max|g| {np.abs(t).max():.3e} ours-f64 {e:.3e} rel {e / (np.abs(t).max() + 1e-30):.2e}")


if "small" in which:
    z = np.load(os.path.join(ROOT, "tests", "golden", "learner_small.npz"))
    mcfg = learner_model_cfg()
    K = int(z["K"])
    start = init_state_dict(mcfg, int(z["seed"]))
    ln = Learner(mcfg, start, K=K)
    for s in (1, 2):
        if s == 2:
            start = {k[len("s1/param/"):]: z[k] for k in z.files if k.startswith("s1/param/")}
            ln.load_state_dict(start)
            ln.load_optimizer_state_dict({"state": {i: {"step": 1.0, "exp_avg": z[f"s1/opt/exp_avg/{k}"],
                                                        "exp_avg_sq": z[f"s1/opt/exp_avg_sq/{k}"]}
                                                    for i, k in enumerate(ln.params)}})
        ring = MinibatchRing(mb_of(z, s))
        print("small", s, "loss", ln.train_minibatch(ring, ring.slots()).cpu().numpy(), float(z[f"s{s}/loss"]))
        report(ln, mcfg, start, mb_of(z, s), K, f"small{s}")
if "full" in which:
    z = np.load(os.path.join(ROOT, "tests", "golden", "learner_full.npz"))
    mcfg = default_config()["model"]
    start = init_state_dict(mcfg, int(z["seed"]))
    ln = Learner(mcfg, start, K=int(z["K"]))
    ring = MinibatchRing(mb_of(z, 1))
    print("full loss", ln.train_minibatch(ring, ring.slots()).cpu().numpy(), float(z["s1/loss"]))
    report(ln, mcfg, start, mb_of(z, 1), int(z["K"]), "full")
if "bf16" in which:
    z = np.load(os.path.join(ROOT, "tests", "golden", "learner_full.npz"))
    mcfg = default_config()["model"]
    ring = MinibatchRing(mb_of(z, 1))
    out = {}
    for dt in ("f32", "bf16"):
        ln = Learner(mcfg, init_state_dict(mcfg, int(z["seed"])), K=int(z["K"]), dtype=dt)
        out[dt] = (ln.train_minibatch(ring, ring.slots()).cpu().numpy(), ln.gradients(),
                   [t.cpu().numpy() for t in ln.last_logits])
    print("bf16 loss", out["bf16"][0], "f32", out["f32"][0])
    for i, key in enumerate(("lr", "lv", "lp")):
        print("  logits", key, "max|diff|", float(np.abs(out["bf16"][2][i] - out["f32"][2][i]).max()))
    for k, g in out["f32"][1].items():
        a, b = g.reshape(-1).double(), out["bf16"][1][k].reshape(-1).double()
        print(f"  {k:45s} cos {float(a @ b / (a.norm() * b.norm() + 1e-30)):.4f} |f32| {float(a.norm()):.3e}"
              f" |bf16| {float(b.norm()):.3e}")
