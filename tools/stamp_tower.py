"""Phase breakdown of tower8_kernel from in-kernel s_memtime stamps (diagnostic build only:
make -C muzero-breakout_amd/csrc tower-stamps -> libmzba_tstamp.so).

  python tools/stamp_tower.py [B] [NBLOCKS] [JSON_OUT]

Runs the plain tower (8-env kernel, random bf16 weights / inputs) 30 times, reads the stamps of the
last launch and prints per-conv medians (over workgroups and waves) of: the k loop split by column
pass (one pass over all three column shifts in the 8-env kernel), the wait at the first barrier, the write-back + second barrier, the
in-kernel clock (s_memtime / s_memrealtime x 100 MHz), and the MFMA-only floor of a conv
(2496 v_mfma_f32_16x16x32_bf16 per wave x 16 cycles). The stamps' own cost perturbs the phases a
little; the shares are what count."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

P, I, LL = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
TST_N, TST_WG = 192, 1024


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 14
    D = ctypes.CDLL(os.path.join(ROOT, "muzero-breakout_amd", "mzba", os.environ.get("TSTAMP_LIB", "libmzba_tstamp.so")))
    D.mzba_tower.argtypes = [P, LL, P, LL, P, P, P, I, I, P, LL, P]
    D.mzba_tower_stamps_read.argtypes = [P, I]
    D.mzba_tower_set_variant.argtypes = [I]
    assert D.mzba_tower_set_variant(2) == 0
    C = 256
    # STAMP_ELEM=1: the fp16 tower (config 5's dynamics net: fp16 LDS images, weights, MFMA) through
    # mzba_tower_fused with no prologue / epilogue; STAMP_ELEM=0 the bf16 tower through the same call
    elem = os.environ.get("STAMP_ELEM")
    wdt = torch.float16 if elem == "1" else torch.bfloat16
    g = torch.Generator().manual_seed(0)
    x = torch.rand(B * 20 * C, generator=g).to(torch.bfloat16).cuda()
    wf = (torch.randn(2 * nb * C * 2304 + 8 * 64 * 8, generator=g) * 0.02).to(wdt).cuda()
    b = (torch.randn(2 * nb * C, generator=g) * 0.1).cuda()
    y = torch.empty_like(x)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    if elem is not None:
        from mzba._lib import TowerExt
        D.mzba_tower_fused.argtypes = [P, LL, P, LL, P, P, P, I, I, P, P]
        ext = TowerExt()
        ext.epilogue, ext.elem, ext.plan = 0, int(elem), 2
    for it in range(30):
        if it == 29:
            ev[0].record()
        if elem is not None:
            assert D.mzba_tower_fused(x.data_ptr(), 20 * C, None, 0, y.data_ptr(), wf.data_ptr(), b.data_ptr(), nb, B,
                                      ctypes.byref(ext), st) == 0
        else:
            assert D.mzba_tower(x.data_ptr(), 20 * C, None, 0, y.data_ptr(), wf.data_ptr(), b.data_ptr(), nb, B, None, 0,
                                st) == 0
    ev[1].record()
    torch.cuda.synchronize()
    nwg = (B + 7) // 8
    rows = min(nwg, TST_WG) * 4
    buf = (ctypes.c_ulonglong * (TST_N * rows))()
    assert D.mzba_tower_stamps_read(buf, rows) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(rows, TST_N).astype(np.float64)
    clock = np.median((a[:, TST_N - 1] - a[:, 0]) / (a[:, TST_N - 2] - a[:, TST_N - 3]) * 0.1)  # GHz
    nconv = 2 * nb
    ph = np.zeros((rows, nconv, 6))
    for ci in range(nconv):
        s = a[:, 2 + 6 * ci: 8 + 6 * ci]
        nxt = a[:, 2 + 6 * (ci + 1)] if ci + 1 < nconv else a[:, TST_N - 1]
        ph[:, ci, 0] = s[:, 1] - s[:, 0]  # bias init (+ the dx 0 pass of a two-pass k loop)
        ph[:, ci, 1] = s[:, 2] - s[:, 1]  # (empty since the passes were merged)
        ph[:, ci, 2] = s[:, 3] - s[:, 2]  # the one-pass k loop (or the dx -1 / +1 pass)
        ph[:, ci, 3] = s[:, 4] - s[:, 3]  # first barrier wait
        ph[:, ci, 4] = s[:, 5] - s[:, 4]  # write-back + second barrier
        ph[:, ci, 5] = nxt - s[:, 5]      # to the next conv's start
    med = np.median(ph[:, 1:-1, :], axis=(0, 1))  # interior convs
    conv = float(med.sum())
    floor = 2496 * 16
    out = {"B": B, "nblocks": nb, "elem": {"1": "fp16", "0": "bf16"}.get(elem, "bf16 (mzba_tower)"), "launch_us": ev[0].elapsed_time(ev[1]) * 1e3, "clock_ghz": float(clock),
           "cycles_per_conv": conv, "mfma_floor_cycles": floor, "mfma_frac_in_conv": floor / conv,
           "phase_cycles": {"bias init (+ dx0 pass if two-pass)": float(med[0]), "-": float(med[1]),
                            "k loop (one pass; dx-1/+1 pass if two-pass)": float(med[2]),
                            "barrier1_wait": float(med[3]), "writeback+barrier2": float(med[4]),
                            "to_next_conv": float(med[5])},
           "mfma_floor_k_loop": 2496 * 16,
           "staging_cycles": float(np.median(a[:, 1] - a[:, 0])),
           "kernel_cycles_per_wg": float(np.median(a[:, TST_N - 1] - a[:, 0])),
           "wave_skew_at_barrier1": float(np.median(
               np.ptp(a.reshape(-1, 4, TST_N)[:, :, 5 + 6 * 10], axis=1)))}
    # launch timeline from the wave-0 real-time stamps (100 MHz, chip-wide): workgroup start / end
    # relative to the first start, durations, and the span the launch adds beyond its workgroups
    w0 = a.reshape(-1, 4, TST_N)[:, 0, :]
    t0, t1 = w0[:, TST_N - 3] * 10e-3, w0[:, TST_N - 2] * 10e-3  # us
    t1 = t1 - t0.min()
    t0 = t0 - t0.min()
    dur = t1 - t0
    order = np.argsort(t0)
    first, second = order[: len(order) // 2], order[len(order) // 2:]
    out["timeline_us"] = {
        "span": float(t1.max()), "wg_duration_min_med_max": [float(dur.min()), float(np.median(dur)), float(dur.max())],
        "round1_start_spread": float(np.ptp(t0[first])), "round1_end_min_max": [float(t1[first].min()), float(t1[first].max())],
        "round2_start_min_max": [float(t0[second].min()), float(t0[second].max())],
        "round2_end_min_med_max": [float(t1[second].min()), float(np.median(t1[second])), float(t1[second].max())],
        # workgroup i runs on XCD i % 8 (round-robin dispatch): per-XCD median duration and last end
        "xcd_median_duration": [float(np.median(dur[x::8])) for x in range(8)],
        "xcd_last_end": [float(t1[x::8].max()) for x in range(8)],
        "xcd_clock_ghz": [float(np.median(((a.reshape(-1, 4, TST_N)[x::8, 0, TST_N - 1] - a.reshape(-1, 4, TST_N)[x::8, 0, 0])
                                            / (w0[x::8, TST_N - 2] - w0[x::8, TST_N - 3]) * 0.1))) for x in range(8)],
    }
    print(json.dumps(out))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
