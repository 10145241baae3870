"""Representation timing at the acting batch (default B = 4096), same box, alternating: the whole net
(rep input -> scaled root latent) with the 256-channel 16x20 blocks as one mzba_rep_blocks launch vs
one mzba_conv_band_res launch per block, and those kernels alone (3 blocks); HIP events, medians of 20.
usage (GPU box): python tools/ab_repblocks.py [B]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ab_rep import timed, L, MuZeroAgent, default_config, init_state_dict, torch  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    mcfg = default_config()["model"]
    ag = MuZeroAgent(mcfg, dtype="bf16")
    ag.load_state_dict(init_state_dict(mcfg, 0))
    rn = ag.runner(B, 16, 20)
    x = torch.rand(B * 320 * 64, device="cuda").to(torch.bfloat16)
    out = torch.empty(B * 20 * 256, dtype=torch.bfloat16, device="cuda")
    res = {"B": B}
    for on in (True, False, True, False):
        rn.use_rep_blocks = on
        res.setdefault(f"representation_ms_rep_blocks_{on}", []).append(timed(lambda: rn.representation(x, out)))
    rn.use_rep_blocks = True
    C, nb = 256, 3
    g = torch.Generator(device="cuda").manual_seed(1)
    xi = torch.rand(B * 320 * C, device="cuda", generator=g).to(torch.bfloat16)
    o = torch.empty_like(xi)
    t = torch.empty_like(xi)
    w = (torch.randn(2 * nb * C * 9 * C + 8 * 64 * 8, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    bb = torch.zeros(2 * nb * C, device="cuda")
    fl = nb * 2 * 2.0 * B * 320 * C * 9 * C
    one = timed(lambda: L.call("mzba_rep_blocks", L.ptr(xi), L.ptr(o), L.ptr(w), L.ptr(bb), nb, B, L.stream()))

    def per_block():
        a, b_ = xi, t
        for k in range(nb):
            L.call("mzba_conv_band_res", L.ptr(a), L.ptr(w), L.ptr(bb), L.ptr(w), L.ptr(bb), L.ptr(b_), B, 16, 20, C,
                   L.stream())
            a, b_ = b_, (o if b_ is t else t)
    band = timed(per_block)
    res["blocks256x3"] = {"rep_blocks_us": one * 1e3, "band_res_us": band * 1e3,
                          "rep_blocks_frac_of_2500": fl / (one * 1e-3) / 1e12 / 2500,
                          "band_res_frac_of_2500": fl / (band * 1e-3) / 1e12 / 2500}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
