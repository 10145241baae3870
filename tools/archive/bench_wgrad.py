"""Weight-gradient kernel timing (learner): mzba_conv_wgrad per shape and variant (bf16 per-tap
tile kernel vs whole-image kernel; f32), HIP-event median over iterations, FLOP = 2 M Cout Cin taps.
usage: python tools/bench_wgrad.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-breakout_amd")]
import torch  # noqa: E402
from mzba import _lib as L  # noqa: E402

dev = torch.device("cuda")
for (B, H, W, Cin, Cout, ks) in [(512, 4, 5, 256, 256, 3), (512, 4, 5, 264, 256, 3), (512, 8, 10, 256, 256, 3),
                                 (512, 16, 20, 128, 128, 3), (512, 4, 5, 256, 256, 1)]:
    for dt, var in (("bf16", 0), ("bf16", 1), ("f32", 0)):
        tdt = torch.bfloat16 if dt == "bf16" else torch.float32
        x = torch.randn(B, H, W, Cin, device=dev).to(tdt)
        dy = torch.randn(B, H, W, Cout, device=dev).to(tdt)
        dw = torch.zeros(Cout, ks * ks, Cin, device=dev)
        db = torch.zeros(Cout, device=dev)
        nb = L.lib().mzba_conv_wgrad_ws_bytes(B, H, W, Cin, Cout, ks)
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        L.call("mzba_conv_wgrad_set_variant", var)
        ts = []
        for it in range(12):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            L.call("mzba_conv_wgrad", 0 if dt == "f32" else 1, L.ptr(x), L.ptr(dy), B, H, W, Cin, Cout, ks, L.ptr(dw),
                   L.ptr(db), L.ptr(ws), nb, L.stream())
            e1.record()
            torch.cuda.synchronize()
            if it >= 2:
                ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        us = ts[len(ts) // 2]
        fl = 2.0 * B * H * W * Cout * Cin * ks * ks
        print(json.dumps({"shape": [B, H, W, Cin, Cout, ks], "dtype": dt, "variant": var, "us": round(us, 1),
                          "tflops": round(fl / us / 1e6, 1)}), flush=True)
L.call("mzba_conv_wgrad_set_variant", 1)
