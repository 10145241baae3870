"""Pixel-tiled tower (mzba_towerp) vs torch fp32 (small B) and vs tower8 (B = 4096): accuracy and
isolated launch time, same box, alternating. Usage: python tools/bench_towerp.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mzba import _lib as L  # noqa: E402
from mzba.agent import pack_tower_conv  # noqa: E402

C, H, W = 256, 4, 5


def make(B, nblocks, gather, seed):
    g = torch.Generator().manual_seed(seed)
    S1 = 3 if gather else 1
    pool = torch.rand(B, S1, H, W, C, generator=g).to(torch.bfloat16)
    slot = torch.randint(0, S1, (B,), generator=g, dtype=torch.int32)
    ws = [torch.randn(C, C, 3, 3, generator=g) / (C * 9) ** 0.5 for _ in range(2 * nblocks)]
    bs = [torch.randn(C, generator=g) * 0.1 for _ in range(2 * nblocks)]
    wf = np.concatenate([pack_tower_conv(w.numpy()) for w in ws] + [np.zeros(8 * 64 * 8, np.float32)])
    d = dict(pool=pool.cuda(), slot=slot.cuda(), wf=torch.from_numpy(wf).to(torch.bfloat16).cuda(), b=torch.cat(bs).cuda(),
             S1=S1, gather=gather)
    return d, pool, slot, ws, bs


def ref(pool, slot, ws, bs, nblocks):
    x = pool[torch.arange(pool.shape[0]), slot.long()].float().permute(0, 3, 1, 2).cuda()
    bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    for k in range(nblocks):
        w1, w2 = bf(ws[2 * k]).cuda(), bf(ws[2 * k + 1]).cuda()
        t1 = bf(torch.relu(torch.nn.functional.conv2d(x, w1, bs[2 * k].cuda(), padding=1)))
        x = bf(torch.relu(torch.nn.functional.conv2d(t1, w2, bs[2 * k + 1].cuda(), padding=1) + x))
    return x.permute(0, 2, 3, 1)


def launch(d, out, B, nblocks, which):
    sl = L.ptr(d["slot"]) if d["gather"] else None
    if which == "p":
        L.call("mzba_towerp", L.ptr(d["pool"]), d["S1"] * H * W * C, sl, H * W * C, L.ptr(out), L.ptr(d["wf"]),
               L.ptr(d["b"]), nblocks, B, L.stream())
    else:
        L.call("mzba_tower_set_variant", 2)
        L.call("mzba_tower", L.ptr(d["pool"]), d["S1"] * H * W * C, sl, H * W * C, L.ptr(out), L.ptr(d["wf"]),
               L.ptr(d["b"]), nblocks, B, None, 0, L.stream())
        L.call("mzba_tower_set_variant", 0)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    # accuracy vs torch fp32 (bf16 weights and intermediates), partial last workgroup included
    for B, nb, gather in [(16, 1, False), (40, 2, True), (256, 3, True)]:
        d, pool, slot, ws, bs = make(B, nb, gather, B + nb)
        out = torch.empty(B, H, W, C, dtype=torch.bfloat16, device="cuda")
        launch(d, out, B, nb, "p")
        torch.cuda.synchronize()
        r = ref(pool, slot, ws, bs, nb)
        err = (out.float() - r).abs().max().item() / max(1.0, r.abs().max().item())
        print(json.dumps({"check": "vs_torch_fp32", "B": B, "nblocks": nb, "gather": gather, "rel_err": err}), flush=True)
    # timing at the headline batch, 14 blocks, alternating with tower8 (plan 2)
    B, nb = 4096, 14
    d, pool, slot, ws, bs = make(B, nb, True, 7)
    outp = torch.empty(B, H, W, C, dtype=torch.bfloat16, device="cuda")
    out8 = torch.empty_like(outp)
    launch(d, outp, B, nb, "p")
    launch(d, out8, B, nb, "8")
    torch.cuda.synchronize()
    dif = (outp.float() - out8.float()).abs()
    print(json.dumps({"check": "towerp_vs_tower8", "B": B, "max_abs": dif.max().item(), "mean_abs": dif.mean().item(),
                      "ref_max": out8.float().abs().max().item()}), flush=True)
    fl = 2.0 * B * 20 * C * 2304 * 2 * nb
    for rep in range(reps):
        for which in ("8", "p"):
            o = outp if which == "p" else out8
            for _ in range(3):
                launch(d, o, B, nb, which)
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
            for e0, e1 in ev:
                e0.record(); launch(d, o, B, nb, which); e1.record()
            torch.cuda.synchronize()
            ms = float(np.median([a.elapsed_time(c) for a, c in ev]))
            print(json.dumps({"kernel": "towerp" if which == "p" else "tower8<0,2>", "rep": rep, "B": B, "nblocks": nb,
                              "us": ms * 1e3, "tflops_alg": fl / (ms * 1e-3) / 1e12}), flush=True)


if __name__ == "__main__":
    main()
