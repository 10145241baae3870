"""Representation net timing at the acting batch (default B = 4096): the whole net (rep input ->
scaled root latent, one NetRunner.representation call) with the 16x20 residual blocks as one launch
each (use_band_res) and as two band-conv launches, and the block kernel alone at C = 256 / 128 vs its
two band convs; HIP events, medians of 20. usage (GPU box): python tools/ab_rep.py [B]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mzba import _lib as L  # noqa: E402
from mzba.agent import MuZeroAgent  # noqa: E402
from mzba.config import default_config  # noqa: E402
from mzba.weights import init_state_dict  # noqa: E402


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    mcfg = default_config()["model"]
    ag = MuZeroAgent(mcfg, dtype="bf16")
    ag.load_state_dict(init_state_dict(mcfg, 0))
    rn = ag.runner(B, 16, 20)
    x = torch.rand(B * 320 * 64, device="cuda").to(torch.bfloat16)
    out = torch.empty(B * 20 * 256, dtype=torch.bfloat16, device="cuda")
    res = {"B": B}
    for fused in (True, False, True, False):
        rn.use_band_res = fused
        res.setdefault(f"representation_ms_band_res_{fused}", []).append(timed(lambda: rn.representation(x, out)))
    rn.use_band_res = True
    for C in (256, 128):
        g = torch.Generator(device="cuda").manual_seed(C)
        xi = torch.rand(B * 320 * C, device="cuda", generator=g).to(torch.bfloat16)
        t = torch.empty_like(xi)
        o = torch.empty_like(xi)
        w = (torch.randn(C * 9 * C + 8 * 64 * 8, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
        bb = torch.zeros(C, device="cuda")
        fl = 2 * 2.0 * B * 320 * C * 9 * C
        one = timed(lambda: L.call("mzba_conv_band_res", L.ptr(xi), L.ptr(w), L.ptr(bb), L.ptr(w), L.ptr(bb), L.ptr(o),
                                   B, 16, 20, C, L.stream()))

        def two_fn():
            L.call("mzba_conv_band", L.ptr(xi), L.ptr(w), L.ptr(bb), None, L.ptr(t), B, 16, 20, C, C, 1, L.stream())
            L.call("mzba_conv_band", L.ptr(t), L.ptr(w), L.ptr(bb), L.ptr(xi), L.ptr(o), B, 16, 20, C, C, 1, L.stream())
        two = timed(two_fn)
        res[f"block{C}"] = {"band_res_us": one * 1e3, "two_band_us": two * 1e3,
                            "band_res_frac_of_2500": fl / (one * 1e-3) / 1e12 / 2500,
                            "two_band_frac_of_2500": fl / (two * 1e-3) / 1e12 / 2500}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
