"""conv_big_bf16_kernel vs conv_igemm (mzba_conv2d variant 1 / 0) on config 3's large convs:
21x21 latent 3x3 256->256 (B = 4096), 42x42 / 84x84 representation convs. HIP-event median."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-breakout_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mzba import _lib as L  # noqa: E402

dev = torch.device("cuda")
for (B, H, W, Cin, Cout, ks) in [(4096, 21, 21, 256, 256, 3), (1024, 42, 42, 256, 256, 3), (512, 84, 84, 128, 256, 3)]:
    x = torch.randn(B * H * W * Cin, device=dev).to(torch.bfloat16)
    w = (torch.randn(Cout * ks * ks * Cin, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.zeros(Cout, device=dev)
    out = torch.empty(B * H * W * Cout, dtype=torch.bfloat16, device=dev)
    fl = 2.0 * B * H * W * Cout * Cin * ks * ks
    for v in (1, 0):
        L.call("mzba_conv2d_set_variant", v)
        ts = []
        for it in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            L.call("mzba_conv2d", 1, L.ptr(x), H * W * Cin, None, 0, L.ptr(w), L.ptr(b), None, None, 0, L.ptr(out),
                   L.ptr(out), B, H, W, Cin, Cout, ks, 1, L.stream())
            e1.record()
            torch.cuda.synchronize()
            if it >= 2:
                ts.append(e0.elapsed_time(e1))
        ms = float(np.median(ts))
        print(json.dumps({"shape": [B, H, W, Cin, Cout, ks], "variant": v, "us": round(ms * 1e3, 1),
                          "tflops": round(fl / ms / 1e9, 1)}), flush=True)
    L.call("mzba_conv2d_set_variant", 1)
