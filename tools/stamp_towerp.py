"""Phase breakdown of towerp_kernel (plan 4) from in-kernel s_memtime stamps (diagnostic build only:
make -C muzero-breakout_amd/csrc towerp-stamps -> libmzba_pstamp.so, loaded through MZBA_LIB).

  MZBA_LIB=$PWD/muzero-breakout_amd/mzba/libmzba_pstamp.so python tools/stamp_towerp.py [MODE] [JSON_OUT]

MODE plain: the 14-block tower at B = 4096 (random bf16 weights); dyn / pred: the fused dynamics /
prediction step of the random-init reference nets through the agent's runner (B = 4096). 30 launches,
the stamps of the last one. Per conv (medians over workgroups and waves, the first and last conv
excluded): pass 0 k loop, pack + pass-1 init + pass 1 k loop, first-barrier wait, write-back + second
barrier; the MFMA-only floor of a pass (2 080 v_mfma_f32_16x16x32_bf16 x 16 cycles); staging, epilogue
phases and the in-kernel clock (s_memtime / s_memrealtime x 100 MHz). The stamps' own cost perturbs
the phases a little; the shares are what count."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mzba import _lib as L  # noqa: E402

PST_N, PST_WG = 192, 256
C = 256


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
    B, nb = 4096, 14
    D = L.lib()
    D.mzba_towerp_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    g = torch.Generator().manual_seed(0)
    if mode == "plain":
        x = torch.rand(B * 20 * C, generator=g).to(torch.bfloat16).cuda()
        wf = (torch.randn(2 * nb * C * 2304 + 8 * 64 * 8, generator=g) * 0.02).to(torch.bfloat16).cuda()
        b = (torch.randn(2 * nb * C, generator=g) * 0.1).cuda()
        y = torch.empty_like(x)
        launch = lambda: L.call("mzba_towerp", L.ptr(x), 20 * C, None, 0, L.ptr(y), L.ptr(wf), L.ptr(b), nb, B,  # noqa: E731
                                L.stream())
        pro = False
    else:
        from mzba.agent import MuZeroAgent
        from mzba.config import default_config
        from mzba.weights import init_state_dict
        mcfg = default_config()["model"]
        ag = MuZeroAgent(mcfg, dtype="bf16")
        ag.load_state_dict(init_state_dict(mcfg, 7))
        L.call("mzba_tower_set_variant", 4)
        rn = ag.runner(B, 16, 20)
        L.call("mzba_tower_set_variant", 0)
        assert rn.tower_plan == 4
        n = 20 * C
        src = torch.rand(B, n, generator=g).to(torch.bfloat16).cuda()
        act = torch.randint(0, 3, (B,), generator=g, dtype=torch.int32).cuda()
        o = torch.empty(B, n, dtype=torch.bfloat16, device="cuda")
        f = lambda *s: torch.empty(s, device="cuda")  # noqa: E731
        r, rl, pi, v, plg, vlg = f(B), f(B, 11), f(B, 3), f(B), f(B, 3), f(B, 11)
        if mode == "dyn":
            launch = lambda: rn.dynamics(src, act, o, r, rl)  # noqa: E731
        else:
            launch = lambda: rn.prediction(src, pi, v, plg, vlg)  # noqa: E731
        pro = mode == "dyn"
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    nrow = PST_WG * 4
    prev = np.zeros((nrow, PST_N), dtype=np.uint64)
    for it in range(30):
        if it == 29:
            torch.cuda.synchronize()
            assert D.mzba_towerp_stamps_read(prev.ctypes.data, nrow) == 0  # launch 28's stamps
            ev[0].record()
        launch()
    ev[1].record()
    torch.cuda.synchronize()
    wall_us = ev[0].elapsed_time(ev[1]) * 1e3
    st = np.zeros((nrow, PST_N), dtype=np.uint64)
    assert D.mzba_towerp_stamps_read(st.ctypes.data, nrow) == 0
    st = st.astype(np.int64)
    nconv = 2 * nb + (1 if pro else 0)
    floor = 2080 * 16

    def med(a, b_):
        return float(np.median(st[:, b_] - st[:, a]))
    rows = []
    for ci in range(1, nconv - 1):
        k = 2 + 5 * ci
        rows.append({"pass0": st[:, k + 1] - st[:, k], "pass1": st[:, k + 2] - st[:, k + 1],
                     "barrier1": st[:, k + 3] - st[:, k + 2], "writeback": st[:, k + 4] - st[:, k + 3],
                     "conv": st[:, k + 5] - st[:, k] if ci + 1 < nconv else st[:, k + 4] - st[:, k]})
    out = {k: float(np.median(np.concatenate([r[k] for r in rows]))) for k in rows[0]}
    # conv1 (the write-back lifts the residual out of the image first) vs conv2 of a block
    c1 = [r for ci, r in zip(range(1, nconv - 1), rows) if (ci - (1 if pro else 0)) % 2 == 0]
    c2 = [r for ci, r in zip(range(1, nconv - 1), rows) if (ci - (1 if pro else 0)) % 2 == 1]
    by_type = {nm: {k: float(np.median(np.concatenate([r[k] for r in rr]))) for k in rows[0]} for nm, rr in
               (("conv1", c1), ("conv2", c2))}
    clk = (st[:, PST_N - 1] - st[:, 0]) / np.maximum(1, st[:, PST_N - 2] - st[:, PST_N - 3]) * 0.1  # GHz
    res = {"mode": mode, "B": B, "nblocks": nb, "per_conv_median_cycles": out, "by_conv_type": by_type,
           "mfma_floor_per_pass": floor,
           "conv_frac_of_floor": 2 * floor / out["conv"],
           "staging": med(0, 1), "first_conv_start": med(1, 2),
           "tower_end_to_exit": med(2 + 5 * nconv - 1, PST_N - 1),
           "kernel_cycles": med(0, PST_N - 1), "clock_ghz_median": float(np.median(clk)),
           "launch_wall_us": wall_us,
           "realtime_span_us": float((st[:, PST_N - 2].max() - st[:, PST_N - 3].min()) / 100.0)}
    # per-workgroup spread (s_memrealtime, 100 MHz): dispatch skew of the entries, each workgroup's
    # duration, the tail of the exits; and whether the slow workgroups are the same in two launches (a
    # systematic tail — slower CUs or XCDs — survives a persistent kernel, a random one averages out)
    def wg(stamps):
        s_ = stamps.astype(np.int64).reshape(PST_WG, 4, PST_N)
        ent, ext = s_[:, :, PST_N - 3].min(1), s_[:, :, PST_N - 2].max(1)
        return (ent - ent.min()) / 100.0, (ext - ent.min()) / 100.0, (ext - ent) / 100.0
    ent, ext, dur = wg(st)
    _, _, dur0 = wg(prev)
    pc = lambda a: {f"p{q}": float(np.percentile(a, q)) for q in (0, 50, 90, 99, 100)}  # noqa: E731
    xcd = [float(np.mean(dur[i::8])) for i in range(8)]
    # the same per XCD in core cycles (s_memtime, wave 0) and the clock they imply: equal cycles at
    # different durations = the XCDs' clocks differ; different cycles = memory-side differences
    cyc = (st.astype(np.int64).reshape(PST_WG, 4, PST_N)[:, 0, PST_N - 1] - st.astype(np.int64).reshape(PST_WG, 4, PST_N)[:, 0, 0])
    xcd_cyc = [float(np.mean(cyc[i::8])) for i in range(8)]
    xcd_clk = [c / d / 1e3 for c, d in zip(xcd_cyc, xcd)]
    res["workgroups"] = {"entry_skew_us": pc(ent), "duration_us": pc(dur), "exit_us": pc(ext),
                         "duration_by_xcd_us": xcd, "cycles_by_xcd": xcd_cyc, "clock_ghz_by_xcd": xcd_clk,
                         "duration_corr_with_previous_launch": float(np.corrcoef(dur, dur0)[0, 1]),
                         "previous_launch_duration_us": pc(dur0)}
    if mode != "plain":
        e = [160, 161, 162, 163, 164]
        last = 2 + 5 * (nconv - 1) + 4
        res["epilogue"] = {f"{a}->{b_}": med(a, b_) for a, b_ in zip([last] + e[:-1], e) if st[:, b_].any()}
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
