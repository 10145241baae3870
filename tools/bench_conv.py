"""Micro-benchmark of the conv kernels on the MI355X (isolated launches, HIP events)."""
import os
import sys
import json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mzba import _lib as L  # noqa: E402


def run(B, H, W, Cin, Cout, ks, kind, iters=50):
    x = torch.randn(B * H * W * Cin, device="cuda").to(torch.bfloat16)
    out = torch.empty(B * H * W * Cout, device="cuda", dtype=torch.bfloat16)
    K = ks * ks * Cin
    w = (torch.randn(Cout * K + 8 * 64 * 8, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.zeros(Cout, device="cuda")

    wt = None
    if kind == "band":
        wt = (torch.randn(Cout * K + 8 * 64 * 8, device="cuda") * 0.02).to(torch.bfloat16)

    def launch():
        if kind == "band":
            L.call("mzba_conv_band", L.ptr(x), L.ptr(wt), L.ptr(b), None, L.ptr(out), B, H, W, Cin, Cout, 1, L.stream())
        elif kind == "lat":
            L.call("mzba_conv_lat", L.ptr(x), H * W * Cin, None, 0, L.ptr(w), L.ptr(b), None, None, 0, L.ptr(x)
                   if Cin == Cout else None, L.ptr(out), B, H, W, Cin, Cout, ks, 1, L.stream())
        else:
            L.call("mzba_conv2d", 1, L.ptr(x), H * W * Cin, None, 0, L.ptr(w), L.ptr(b), None, None, 0, L.ptr(x)
                   if Cin == Cout else None, L.ptr(out), B, H, W, Cin, Cout, ks, 1, L.stream())
    for _ in range(5):
        launch()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for e0, e1 in ev:
        e0.record(); launch(); e1.record()
    torch.cuda.synchronize()
    ms = np.median([a.elapsed_time(c) for a, c in ev])
    fl = 2.0 * B * H * W * Cout * K
    return {"kind": kind, "B": B, "HW": (H, W), "Cin": Cin, "Cout": Cout, "ks": ks, "us": ms * 1e3,
            "tflops": fl / (ms * 1e-3) / 1e12}


def run_tower(B, nblocks, iters=20, variant=0):
    C = 256
    L.call("mzba_tower_set_variant", variant)
    nb = L.lib().mzba_tower_ws_bytes(B)
    ws = torch.zeros(max(nb, 16), dtype=torch.uint8, device="cuda")
    x = torch.randn(B * 20 * C, device="cuda").to(torch.bfloat16)
    out = torch.empty_like(x)
    wf = (torch.randn(2 * nblocks * C * 2304 + 8 * 64 * 8, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.zeros(2 * nblocks * C, device="cuda")


    def launch():
        L.call("mzba_tower", L.ptr(x), 20 * C, None, 0, L.ptr(out), L.ptr(wf), L.ptr(b), nblocks, B, L.ptr(ws), nb,
               L.stream())
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for e0, e1 in ev:
        e0.record(); launch(); e1.record()
    torch.cuda.synchronize()
    ms = np.median([a.elapsed_time(c) for a, c in ev])
    fl = 2.0 * B * 20 * C * 2304 * 2 * nblocks
    L.call("mzba_tower_set_variant", 0)
    return {"kind": "tower", "variant": variant, "B": B, "nblocks": nblocks, "us": ms * 1e3, "us_per_conv": ms * 1e3 / (2 * nblocks),
            "tflops": fl / (ms * 1e-3) / 1e12}


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "tower":
        for s in [(1024, 1), (1024, 14), (2048, 14), (4096, 14)]:
            for v in (1, 2, 3):
                print(json.dumps(run_tower(*s, variant=v)))
        print(json.dumps(run(1024, 4, 5, 256, 256, 3, "lat")))
        sys.exit(0)
    shapes = [(1024, 4, 5, 256, 256, 3), (1024, 4, 5, 256, 256, 1), (1024, 8, 10, 256, 256, 3),
              (1024, 16, 20, 256, 256, 3), (1024, 16, 20, 128, 128, 3), (1024, 16, 20, 64, 128, 3),
              (1024, 16, 20, 128, 256, 3)]
    if len(sys.argv) > 1 and sys.argv[1] == "rep":
        for s in shapes[2:]:
            for kind in ("gen", "lat", "band"):
                if kind == "lat" and not L.lib().mzba_conv_lat_supported(*s[1:]):
                    continue
                if kind == "band" and not L.lib().mzba_conv_band_supported(*s[1:]):
                    continue
                print(json.dumps(run(*s, kind)))
        sys.exit(0)
    for s in shapes:
        for kind in ("gen", "lat"):
            print(json.dumps(run(*s, kind)))
