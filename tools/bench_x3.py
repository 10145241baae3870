"""Isolated timing of the f32 parity path's latent conv forms at the acting loop's shape (B = 4096, 4x5 latent,
256 -> 256, 3x3): the split-fp16 x3 form (mzba_conv_x3_ex, round 6) and the split-bf16 x6 pixel-tiled form
(mzba_conv_x6_ex, variant 3), plain and with a residual. HIP events around 20 launches after 3 warm-up launches.
One JSON line per (form, residual); `frac` against the form's own ceiling (x3: 2500 / 3 TF, x6: 2500 / 6) in
algorithmic FLOPs (the reference's Conv2d(padding=1) counts the padding taps). Output checksums (f32 bit patterns,
position-weighted) compare builds: equal = bit-identical. A same-box A/B alternates processes with MZBA_LIB.
  python tools/bench_x3.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "muzero-breakout_amd"))
from mzba import _lib as L  # noqa: E402
from mzba.agent import split_pack_x3, split_pack_x6  # noqa: E402


def timeit(fn, n=20, warm=3):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    tag = os.environ.get("MZBA_LIB", "libmzba.so").rsplit("/", 1)[-1]
    dev = torch.device("cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    B, H, W, C = 4096, 4, 5, 256
    x = torch.rand(B, H, W, C, generator=g, device=dev)
    w = (torch.randn(C, 9 * C, generator=g, device=dev) / 48.0).cpu().numpy()
    wx6 = split_pack_x6(w, C, 3, C).to(dev)
    wx3, wsc = split_pack_x3(w, C, 3, C)
    wx3, wsc = wx3.to(dev), wsc.to(dev)
    b = torch.randn(C, generator=g, device=dev)
    out = torch.empty(B, H, W, C, device=dev)
    fl = 2.0 * B * H * W * C * 9 * C
    L.call("mzba_conv_x6_set_variant", 3)
    for rep in range(2):
        for form in ("x3", "x3nopipe", "x3dual", "x6"):
            if form.startswith("x3") and hasattr(L.lib(), "mzba_conv_x3_set_pipe"):
                L.call("mzba_conv_x3_set_pipe", {"x3": 1, "x3nopipe": 0, "x3dual": 2}[form])
            for res in (None, x):
                if form.startswith("x3"):
                    fn = lambda: L.call("mzba_conv_x3_ex", L.ptr(x), H * W * C, None, 0, L.ptr(wx3), L.ptr(wsc), L.ptr(b),  # noqa
                                        None, None, 0, L.ptr(res), L.ptr(out), B, H, W, C, C, 3, 1, L.stream())
                else:
                    fn = lambda: L.call("mzba_conv_x6_ex", L.ptr(x), H * W * C, None, 0, L.ptr(wx6), L.ptr(b),  # noqa
                                        None, None, 0, L.ptr(res), L.ptr(out), B, H, W, C, C, 3, 1, L.stream())
                ms = timeit(fn)
                h = out.view(torch.int32).flatten().to(torch.int64)
                ck = int((h * (torch.arange(h.numel(), device=dev) % 65521 + 1)).sum().item())
                peak = 2500.0 / (3 if form.startswith("x3") else 6)
                print(json.dumps({"lib": tag, "form": form, "residual": res is not None, "rep": rep, "ms": ms,
                                  "tflops": fl / ms / 1e9, "peak": peak, "frac": fl / ms / 1e9 / peak,
                                  "checksum": ck}), flush=True)
    L.call("mzba_conv_x6_set_variant", 2)
    if hasattr(L.lib(), "mzba_conv_x3_set_pipe"):
        L.call("mzba_conv_x3_set_pipe", 1)


if __name__ == "__main__":
    main()
