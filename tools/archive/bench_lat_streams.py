"""Learner latent layer chain (conv_lat B=512 3x3 256->256 + train-mode BN stats/apply) as one
stream vs two independent chains on two streams (the prediction and dynamics towers of one
unroll step are independent). HIP-event wall time of the whole batch of launches, median of 5."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-breakout_amd")]
import json  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mzba import _lib as L  # noqa: E402
from mzba.agent import pack_lat  # noqa: E402

dev = torch.device("cuda")
B, H, W, C, N = 512, 4, 5, 256, 28
M = B * H * W
w = torch.randn(C, C, 3, 3) / (C * 9) ** 0.5
wf = torch.from_numpy(pack_lat(w.permute(0, 2, 3, 1).reshape(C, -1).numpy(), C, 3, C)).to(torch.bfloat16).to(dev)
bias = torch.zeros(C, device=dev)
gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)


def chain(x, n, bn):
    ws = torch.empty(((M + 63) // 64) * C * 8 + 12 * C, dtype=torch.uint8, device=dev)
    st = torch.empty(4, C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    for _ in range(n):
        t = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
        L.call("mzba_conv_lat", L.ptr(x), H * W * C, None, 0, L.ptr(wf), L.ptr(bias), None, None, 0, None, L.ptr(t),
               B, H, W, C, C, 3, 0, L.stream())
        if bn:
            L.call("mzba_bn_stats", 1, L.ptr(t), M, C, 1e-5, 0.1, L.ptr(gamma), L.ptr(beta), L.ptr(st), L.ptr(rm),
                   L.ptr(rv), L.ptr(ws), ws.numel(), L.stream())
            y = torch.empty_like(t)
            L.call("mzba_bn_apply", 1, L.ptr(t), L.ptr(st), None, 1, L.ptr(y), M, C, L.stream())
            t = y
        x = t
    return x


x0 = torch.randn(M, C, device=dev).to(torch.bfloat16)
x1 = torch.randn(M, C, device=dev).to(torch.bfloat16)
side = torch.cuda.Stream()
for bn in (False, True):
    res = {}
    for mode in ("one_stream", "two_streams"):
        ts = []
        for it in range(7):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if mode == "one_stream":
                chain(x0, N, bn)
                chain(x1, N, bn)
            else:
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    chain(x1, N, bn)
                chain(x0, N, bn)
                torch.cuda.current_stream().wait_stream(side)
            e1.record()
            torch.cuda.synchronize()
            if it >= 2:
                ts.append(e0.elapsed_time(e1) * 1e3)
        res[mode] = float(np.median(ts))
    print(json.dumps({"bn": bn, "convs": 2 * N, **{k: round(v, 1) for k, v in res.items()},
                      "us_per_conv_one": round(res["one_stream"] / (2 * N), 2),
                      "us_per_conv_two": round(res["two_streams"] / (2 * N), 2)}), flush=True)
