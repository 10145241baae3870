"""Phase breakdown of conv_lat from in-kernel s_memtime stamps (diagnostic build only).
`python tools/stamp_conv.py [variants|ablate|learner|mfma|zrows|libs TAG...]`. Stamps: 0 entry, 1 after staging barrier, 3 wave0 after main loop (7 = wave 4), 4 after the
post-loop barrier, 5 end. Shares are what count (the stamps' fences perturb timing)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

P, I, LL = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong


def load(tag):
    D = ctypes.CDLL(os.path.join(ROOT, "muzero-breakout_amd", "mzba", f"libmzba_diag{tag}.so"))
    D.mzba_conv_lat.argtypes = [P, LL, P, LL, P, P, P, P, I, P, P, I, I, I, I, I, I, I, P]
    D.mzba_lat_stamps_read.argtypes = [P, I]
    D.mzba_conv_lat_set_variant.argtypes = [I]
    D.mzba_conv_lat_bn_chunks.argtypes = [I, I, I, I, I, I, P, P]
    return D


def run(D, B, H, W, Cin, Cout, ks, res=True):
    x = torch.randn(B * H * W * Cin, device="cuda").to(torch.bfloat16)
    out = torch.empty(B * H * W * Cout, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(Cout * ks * ks * Cin + 8 * 64 * 8, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.zeros(Cout, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for it in range(40):
        if it == 20:
            e0.record()
        rc = D.mzba_conv_lat(x.data_ptr(), H * W * Cin, None, 0, w.data_ptr(), b.data_ptr(), None, None, 0,
                             x.data_ptr() if res else None, out.data_ptr(), B, H, W, Cin, Cout, ks, 1, st)
        assert rc == 0
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    nch, rpc = ctypes.c_int(), ctypes.c_int()
    assert D.mzba_conv_lat_bn_chunks(B, H, W, Cin, Cout, ks, ctypes.byref(nch), ctypes.byref(rpc)) == 0
    nblk = nch.value * ((Cout + 127) // 128)
    buf = (ctypes.c_ulonglong * (8 * nblk))()
    D.mzba_lat_stamps_read(buf, nblk)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(nblk, 8).astype(np.float64)
    t0 = a[:, 0].min()
    rel = a - t0
    ph = {"stage": np.median(a[:, 1] - a[:, 0]), "loop_w0": np.median(a[:, 3] - a[:, 1]),
          "loop_w4": np.median(a[:, 7] - a[:, 1]), "wait_barrier": np.median(a[:, 4] - a[:, 3]),
          "epilogue": np.median(a[:, 5] - a[:, 4]), "total_block": np.median(a[:, 5] - a[:, 0]),
          "launch_spread(start max-min)": float(rel[:, 0].max()), "end_max": float(rel[:, 5].max()),
          "us_per_launch": us, "workgroups": nblk}
    return {k: float(v) for k, v in ph.items()}


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "variants"
    if which == "libs":  # diagnostic builds named on the command line (base = libmzba_diag.so), alternated
        tags = ["" if t == "base" else t for t in sys.argv[2:]]
        for rep in range(2):
            for tag in tags:
                D = load(tag)
                for v in (0, 2):
                    assert D.mzba_conv_lat_set_variant(v) == 0
                    for s in [(512, 4, 5, 256, 256, 3), (1024, 4, 5, 256, 256, 3)]:
                        print(json.dumps({"lib": "libmzba_diag%s.so" % tag, "rep": rep, "lat_variant": v, "shape": s,
                                          "cycles": run(D, *s)}), flush=True)
    elif which == "zrows":  # a 16-row zero block (the A/B build of profiles/r05/lat_zero_block, LAT_ZROWS=16) vs one
        # shared zero row (libmzba_diag_z1.so, LAT_ZROWS=1)
        for rep in range(2):
            for tag in ("_z1", ""):
                D = load(tag)
                for v in (0, 2):
                    assert D.mzba_conv_lat_set_variant(v) == 0
                    for s in [(512, 4, 5, 256, 256, 3), (1024, 4, 5, 256, 256, 3)]:
                        print(json.dumps({"zero_rows": 1 if tag else 16, "rep": rep, "lat_variant": v, "shape": s,
                                          "cycles": run(D, *s)}), flush=True)
    elif which == "mfma":  # 16x16x32 vs 32x32x16 MFMAs at the learner's shapes, alternated (needs the A/B build of
        # profiles/r05/lat_mfma16/conv_lat_mfma16_rejected.patch: mzba_conv_lat_set_mfma)
        D = load("")
        D.mzba_conv_lat_set_mfma.argtypes = [I]
        for rep in range(2):
            for mf in (32, 16):
                assert D.mzba_conv_lat_set_mfma(mf) == 0
                for v in (0, 2):
                    assert D.mzba_conv_lat_set_variant(v) == 0
                    for s in [(512, 4, 5, 256, 256, 3), (1024, 4, 5, 256, 256, 3)]:
                        print(json.dumps({"mfma": mf, "rep": rep, "lat_variant": v, "shape": s, "cycles": run(D, *s)}),
                              flush=True)
    elif which == "learner":  # the learner's B = 512 latent conv: 3-row (variant 0) and 5-row (2) tiles
        for tag, name in (("", "full"), ("_a1", "hot 8KB weights"), ("_a2", "no LDS A reads"), ("_a3", "no MFMA")):
            D = load(tag)
            for v in (0, 2):
                assert D.mzba_conv_lat_set_variant(v) == 0
                for s in [(512, 4, 5, 256, 256, 3), (1024, 4, 5, 256, 256, 3)]:
                    print(json.dumps({"variant": name, "lat_variant": v, "shape": s, "cycles": run(D, *s)}), flush=True)
    elif which == "ablate":
        for tag, name in (("", "full"), ("_a1", "hot 8KB weights"), ("_a2", "no LDS A reads"), ("_a3", "no MFMA")):
            D = load(tag)
            for s in [(1024, 4, 5, 256, 256, 3), (1024, 4, 5, 256, 256, 1)]:
                print(json.dumps({"variant": name, "shape": s, "cycles": run(D, *s)}))
    else:
        D = load("")
        for v, name in ((0, "8w ring8"), (1, "4w 2ct/wave")):
            assert D.mzba_conv_lat_set_variant(v) == 0
            for s in [(1024, 4, 5, 256, 256, 3), (4096, 4, 5, 256, 256, 3)]:
                print(json.dumps({"variant": name, "shape": s, "cycles": run(D, *s)}))
