"""Phase breakdown of band_conv_kernel (representation convs at 16x20) from in-kernel s_memtime stamps
(diagnostic build only: make -C muzero-breakout_amd/csrc band-stamps -> libmzba_bstamp.so).

  python tools/stamp_band.py [B] [XT] [JSON_OUT]     (XT = 0: the residual-block kernel, mzba_conv_band_res)

Per (Cin, Cout) of the representation: runs the conv 20 times (random bf16 weights / inputs, residual
when Cin == Cout), reads the stamps of the last launch and prints median cycles per phase (band staging,
k loop, residual staging, epilogue to LDS, stores), the in-kernel clock, the MFMA-only floor of the k
loop (MFMAs per wave x 16 cycles) and the launch's wall time."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402
import torch  # noqa: E402

P, I = ctypes.c_void_p, ctypes.c_int
BST_N, BST_WG = 8, 8192


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    xt = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    D = ctypes.CDLL(os.path.join(ROOT, "muzero-breakout_amd", "mzba", os.environ.get("BSTAMP_LIB", "libmzba_bstamp.so")))
    D.mzba_conv_band.argtypes = [P, P, P, P, P, I, I, I, I, I, I, P]
    D.mzba_band_stamps_read.argtypes = [P, I]
    D.mzba_conv_band_set_xt.argtypes = [I]
    D.mzba_conv_band_res.argtypes = [P, P, P, P, P, P, I, I, I, I, P]
    blocks = xt == 0  # XT = 0: the residual-block kernel (mzba_conv_band_res: both convs, 10-column bands)
    if not blocks:
        assert D.mzba_conv_band_set_xt(xt) == 0
    res = []
    for cin, cout in (((128, 128), (256, 256)) if blocks else ((64, 128), (128, 128), (128, 256), (256, 256))):
        g = torch.Generator().manual_seed(cin + cout)
        x = torch.rand(B * 320 * cin, generator=g).to(torch.bfloat16).cuda()
        wf = (torch.randn(cout * 9 * cin + 8 * 64 * 8, generator=g) * 0.02).to(torch.bfloat16).cuda()
        b = (torch.randn(cout, generator=g) * 0.1).cuda()
        r = torch.rand(B * 320 * cout, generator=g).to(torch.bfloat16).cuda() if cin == cout else None
        y = torch.empty(B * 320 * cout, dtype=torch.bfloat16, device="cuda")
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for it in range(20):
            if it == 19:
                ev[0].record()
            if blocks:
                assert D.mzba_conv_band_res(x.data_ptr(), wf.data_ptr(), b.data_ptr(), wf.data_ptr(), b.data_ptr(),
                                            y.data_ptr(), B, 16, 20, cin, st) == 0
            else:
                assert D.mzba_conv_band(x.data_ptr(), wf.data_ptr(), b.data_ptr(), r.data_ptr() if r is not None else None,
                                        y.data_ptr(), B, 16, 20, cin, cout, 1, st) == 0
        ev[1].record()
        torch.cuda.synchronize()
        nwg = (2 if blocks else 20 // xt) * B
        rows = min(nwg, BST_WG) * 4
        buf = (ctypes.c_ulonglong * (BST_N * rows))()
        assert D.mzba_band_stamps_read(buf, rows) == 0
        a = np.frombuffer(buf, dtype=np.uint64).reshape(rows, BST_N).astype(np.float64)
        clock = np.median((a[:, 5] - a[:, 0]) / (a[:, 7] - a[:, 6]) * 0.1)
        ph = {"staging": a[:, 1] - a[:, 0], "k_loop": a[:, 2] - a[:, 1], "residual_staging": a[:, 3] - a[:, 2],
              "epilogue_lds": a[:, 4] - a[:, 3], "stores": a[:, 5] - a[:, 4], "total": a[:, 5] - a[:, 0]}
        # zero-pad column taps are computed (the band kernels do not skip them); a block runs conv1 over
        # 12 and conv2 over 10 column tiles
        mfma = ((12 + 10) if blocks else xt) * (cout // 64) * 9 * (cin // 32)
        floor = mfma * 16
        ms = ev[0].elapsed_time(ev[1])
        fl = (2 if blocks else 1) * 2.0 * B * 320 * cout * 9 * cin
        out = {"B": B, "xt": xt, "cin": cin, "cout": cout, "launch_us": ms * 1e3, "tflops": fl / (ms * 1e-3) / 1e12,
               "frac_of_2500": fl / (ms * 1e-3) / 1e12 / 2500, "clock_ghz": float(clock),
               "median_cycles": {k: float(np.median(v)) for k, v in ph.items()},
               "k_loop_mfma_floor_cycles": floor, "k_loop_mfma_frac": floor / float(np.median(ph["k_loop"])),
               "wg_duration_us_median": float(np.median(a[:, 7] - a[:, 6]) * 0.01)}
        print(json.dumps(out), flush=True)
        res.append(out)
    if len(sys.argv) > 3:
        json.dump(res, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
