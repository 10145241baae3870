"""Learner latent weight gradient: K = 5 unrolled uses of one 3x3 256->256 conv at 4x5, B = 512
per use. Immediate (5 x mzba_conv_wgrad, per-tap kernel) vs deferred (one mzba_conv_wgrad_segs,
whole-image kernel: form 1 = pixel rows (round 6); form 2 = pixel rows with 64-co wave tiles, the default;
form 0 = zero-bordered images). Also the
representation's 16x20 / 8x10 shapes as single segments. HIP-event median; FLOP = 2 M Cout Cin 9 over all
segments."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-breakout_amd")]
import torch  # noqa: E402
from mzba import _lib as L  # noqa: E402

dev = torch.device("cuda")
for (nseg, B, H, W, Cin, Cout) in [(5, 512, 4, 5, 256, 256), (5, 512, 4, 5, 264, 256), (5, 512, 4, 5, 256, 128),
                                   (1, 512, 8, 10, 256, 256), (1, 512, 16, 20, 128, 128), (1, 512, 16, 20, 256, 256)]:
    xs = [torch.randn(B, H, W, Cin, device=dev).to(torch.bfloat16) for _ in range(nseg)]
    dys = [torch.randn(B, H, W, Cout, device=dev).to(torch.bfloat16) for _ in range(nseg)]
    dw = torch.zeros(Cout, 9, Cin, device=dev)
    db = torch.zeros(Cout, device=dev)
    nb = L.lib().mzba_conv_wgrad_ws_bytes(nseg * B, H, W, Cin, Cout, 3)
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    xp = (ctypes.c_void_p * nseg)(*[t.data_ptr() for t in xs])
    dp = (ctypes.c_void_p * nseg)(*[t.data_ptr() for t in dys])
    fl = 2.0 * nseg * B * H * W * Cout * Cin * 9
    for mode in ("immediate", "segs_img_form0", "segs_img_form1", "segs_img_form2", "segs_img_form3",
                 "segs_img_form2b", "segs_img_form3b"):
        L.call("mzba_conv_wgrad_set_variant", 2 if mode.startswith("segs_img") else 1)
        L.call("mzba_conv_wgrad_set_form", int(mode[13]) if mode.startswith("segs_img") else 1)
        ts = []
        for it in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if mode == "immediate":
                for i in range(nseg):
                    L.call("mzba_conv_wgrad", 1, L.ptr(xs[i]), L.ptr(dys[i]), B, H, W, Cin, Cout, 3, L.ptr(dw),
                           L.ptr(db), L.ptr(ws), nb, L.stream())
            else:
                L.call("mzba_conv_wgrad_segs", 1, xp, dp, nseg, B, H, W, Cin, Cout, 3, L.ptr(dw), L.ptr(db), L.ptr(ws),
                       nb, L.stream())
            e1.record()
            torch.cuda.synchronize()
            if it >= 2:
                ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        us = ts[len(ts) // 2]
        print(json.dumps({"shape": [nseg, B, H, W, Cin, Cout], "mode": mode, "us": round(us, 1),
                          "tflops": round(fl / us / 1e6, 1)}), flush=True)
L.call("mzba_conv_wgrad_set_variant", 1)
L.call("mzba_conv_wgrad_set_form", 2)
