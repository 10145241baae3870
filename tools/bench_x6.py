"""Same-box A/B of the f32-faithful split-bf16 conv (mzba_conv_x6) wave splits and of the halo conv forms, at the
acting loop's shapes: x6 at the 4x5 latent (B = 4096, the parity path's towers) and 8x10 (the representation
tail), halo at config 3's 21x21 latent (B = 4096). HIP events around 20 launches after 3 warm-up launches,
alternated twice. Prints one JSON line per (kernel, shape, variant). The variant setters
(mzba_conv_x6_set_variant: 3 the pixel-tiled form, 1 the pre-split x6 form; mzba_conv_halo_set_form: 0 the 256-pixel
one-per-CU form, 1 the 128-pixel two-per-CU form; config 3's 21x21 shape, where the default is the 256-pixel form) may be missing from a build; the default then runs once per variant
slot (variant None).
  python tools/bench_x6.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "muzero-breakout_amd"))
from mzba import _lib as L  # noqa: E402


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


def set_variant(name, v):
    """variant setters a library may predate (A/B against an older build, MZBA_LIB_PARTIAL=1)"""
    if hasattr(L.lib(), name):
        L.call(name, v)
        return v
    return None


def main():
    tag = os.environ.get("MZBA_LIB", "libmzba.so").rsplit("/", 1)[-1]
    dev = torch.device("cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    C = 256
    for (B, H, W) in (() if os.environ.get("HALO_ONLY") else ((4096, 4, 5), (4096, 8, 10))):
        x = torch.rand(B, H, W, C, generator=g, device=dev)
        wx = torch.randn(3 * C * 9 * C, generator=g, device=dev).to(torch.bfloat16)
        b = torch.randn(C, generator=g, device=dev)
        out = torch.empty(B, H, W, C, device=dev)
        fl = 2.0 * B * H * W * C * 9 * C * 6
        for rep in range(2):
            for v in ((3, 1) if (H, W) == (4, 5) else (1,)):  # 3: pixel-tiled (round 5), 1: pre-split
                v = set_variant("mzba_conv_x6_set_variant", v)
                ms = timeit(lambda: L.call("mzba_conv_x6", L.ptr(x), L.ptr(wx), L.ptr(b), None, L.ptr(out), B, H, W, C, C, 1,
                                           L.stream()))
                # the x6 roofline: six bf16 MFMAs per f32-faithful product against the dense bf16 peak (algorithmic
                # products, the padding taps included, as the reference's Conv2d(padding=1) counts them)
                print(json.dumps({"lib": tag, "kernel": "conv_x6", "shape": [B, H, W, C], "variant": v, "rep": rep, "ms": ms,
                                  "bf16_tflops": fl / ms / 1e9, "frac_bf16_peak": fl / ms / 1e9 / 2500}), flush=True)
        set_variant("mzba_conv_x6_set_variant", 2)
        del x, wx, out
    if os.environ.get("X6_ONLY"):
        return
    B, H, W = 4096, 21, 21
    x = torch.randn(B, H, W, C, generator=g, device=dev).to(torch.bfloat16)
    wh = torch.randn(C * 9 * C, generator=g, device=dev).to(torch.bfloat16)
    b = torch.randn(C, generator=g, device=dev)
    out = torch.empty(B, H, W, C, dtype=torch.bfloat16, device=dev)
    fl = 2.0 * B * H * W * C * 9 * C
    for rep in range(3):
        for v in (2, 1):  # mzba_conv_halo_set_form (round 6: 2 = 256 pixels one per CU, 1 = 128 pixels two per CU)
            v = set_variant("mzba_conv_halo_set_form", v)
            for res in (x, None):
                ms = timeit(lambda: L.call("mzba_conv_halo", L.ptr(x), L.ptr(wh), L.ptr(b), L.ptr(res), L.ptr(out), B, H, W,
                                           C, C, 1, L.stream()), n=10)
                # output checksum (int16 bit patterns, position-weighted): equal across builds = bit-identical
                h = out.view(torch.int16).flatten().to(torch.int64)
                ck = int((h * (torch.arange(h.numel(), device=dev) % 65521 + 1)).sum().item())
                print(json.dumps({"lib": tag, "kernel": "conv_halo", "shape": [B, H, W, C], "form": v,
                                  "residual": res is not None, "rep": rep, "ms": ms, "tflops": fl / ms / 1e9,
                                  "frac": fl / ms / 1e9 / 2500, "checksum": ck}), flush=True)
    set_variant("mzba_conv_halo_set_waves", 0)


if __name__ == "__main__":
    main()
