"""mzba_rep_blocks (csrc/repblocks.hip): the representation's 256-channel ResidualBlocks at 16x20
(networks.py:73-82, ResidualBlock :19-35) in one launch, one env per workgroup with its whole image
LDS-resident. It adds each accumulator's taps in mzba_conv_band_res's order but starts the accumulators
at bias + residual (towerp_kernel's arithmetic) where the band kernels add them after the taps, so the
two differ by f32 rounding: a plain torch fp32 evaluation of the bf16-rounded operands bounds both with
the tolerance of test_band_res_block_equals_two_band_convs (2e-2 of the tensor's magnitude), and the
whole representation net with and without the kernel agrees within test_rep_tail_vs_torch_fp32's 2e-2
on the [0, 1] scaled latent."""
import numpy as np
import pytest
import torch

from mzba.config import default_config
from mzba.weights import init_state_dict

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"


@pytest.mark.parametrize("B,nblocks", [(5, 1), (3, 3), (300, 3)])
def test_rep_blocks_equal_band_res_launches(B, nblocks):
    from mzba import _lib as L
    from mzba.agent import pack_tower_conv, LAT_PAD_ELEMS
    C = 256
    g = torch.Generator().manual_seed(B + nblocks)
    bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    x = bf(torch.rand(B, C, 16, 20, generator=g))
    ws = [bf(torch.randn(C, C, 3, 3, generator=g) / (C * 9) ** 0.5) for _ in range(2 * nblocks)]
    bs = [torch.randn(C, generator=g) * 0.1 for _ in range(2 * nblocks)]
    pk = lambda w: np.concatenate([pack_tower_conv(w.numpy()), np.zeros(LAT_PAD_ELEMS, np.float32)])  # noqa: E731
    x_d = x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).cuda()
    wall = torch.from_numpy(np.concatenate([pack_tower_conv(w.numpy()) for w in ws] + [np.zeros(LAT_PAD_ELEMS, np.float32)]))
    wall = wall.to(torch.bfloat16).cuda()
    ball = torch.cat(bs).cuda()
    one = torch.full((B, 16, 20, C), float("nan"), device="cuda").to(torch.bfloat16)
    L.call("mzba_rep_blocks", L.ptr(x_d), L.ptr(one), L.ptr(wall), L.ptr(ball), nblocks, B, L.stream())
    # the band path: one mzba_conv_band_res launch per block (operands held: a temporary's memory could
    # be handed to the next temporary before the launch reads it)
    cur = x_d
    for k in range(nblocks):
        w1 = torch.from_numpy(pk(ws[2 * k])).to(torch.bfloat16).cuda()
        w2 = torch.from_numpy(pk(ws[2 * k + 1])).to(torch.bfloat16).cuda()
        b1, b2 = bs[2 * k].cuda(), bs[2 * k + 1].cuda()
        nxt = torch.empty_like(cur)
        L.call("mzba_conv_band_res", L.ptr(cur), L.ptr(w1), L.ptr(b1), L.ptr(w2), L.ptr(b2), L.ptr(nxt), B, 16, 20, C,
               L.stream())
        torch.cuda.synchronize()
        cur = nxt
    torch.cuda.synchronize()
    ref = x
    for k in range(nblocks):
        t = bf(torch.relu(torch.nn.functional.conv2d(ref, ws[2 * k], bs[2 * k], padding=1)))
        ref = bf(torch.relu(torch.nn.functional.conv2d(t, ws[2 * k + 1], bs[2 * k + 1], padding=1) + ref))
    mag = max(1.0, ref.abs().max().item())
    got, band = one.float().cpu().permute(0, 3, 1, 2), cur.float().cpu().permute(0, 3, 1, 2)
    assert torch.isfinite(got).all()
    err, err_band = (got - ref).abs().max().item() / mag, (band - ref).abs().max().item() / mag
    print(f"rep_blocks vs torch fp32 [B={B}, {nblocks} blocks]: {err:.2e} (band_res: {err_band:.2e})")
    assert err < 2e-2, err
    assert err_band < 2e-2, err_band
    # most elements round identically (the sums differ only in where bias and residual join)
    assert (got == band).float().mean().item() > 0.8


@pytest.mark.parametrize("B", [13, 4096])
def test_representation_with_rep_blocks(B):
    """The whole representation net (band stem / 128-channel blocks / widening conv, the 256-channel
    blocks, rep_tail) with the blocks as one mzba_rep_blocks launch vs one band_res launch per block, at
    the acting batch: the scaled root latents within 2e-2 (the [0, 1] latent, as
    test_rep_tail_vs_torch_fp32), and the kernel is what the runner launches by default."""
    from mzba.agent import MuZeroAgent
    mcfg = default_config()["model"]
    ag = MuZeroAgent(mcfg, dtype="bf16")
    ag.load_state_dict(init_state_dict(mcfg, 12))
    assert ag.packed.rep_blocks is not None and ag.packed.rep_blocks["n"] == 3
    rn = ag.runner(B, 16, 20)
    assert rn.use_rep_blocks
    rn.use_rep_trunk = False  # the band stem / 128-channel blocks / widening conv, then the blocks under test
    g = torch.Generator().manual_seed(B)
    xs = torch.rand(B, 64, 16, 20, generator=g).cuda()
    lat = {}
    for on in (True, False):
        rn.use_rep_blocks = on
        lat[on] = ag.create_hidden_state_root(xs).float().cpu()
    rn.use_rep_blocks, rn.use_rep_trunk = True, True
    assert torch.isfinite(lat[True]).all()
    d = (lat[True] - lat[False]).abs().max().item()
    print(f"representation, rep_blocks vs band_res [B={B}]: {d:.2e}")
    assert d < 2e-2, d


def _trunk_case(B, n0, n1, seed):
    """Random BN-folded trunk weights (stem 64 -> 128, n0 blocks at 128, widening 128 -> 256, n1 blocks at
    256), bf16-rounded, and a plain torch fp32 evaluation of them that rounds every layer's output to bf16
    as the kernels store it."""
    g = torch.Generator().manual_seed(seed)
    bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    shapes = [(64, 128)] + [(128, 128)] * (2 * n0) + [(128, 256)] + [(256, 256)] * (2 * n1)
    ws = [bf(torch.randn(co, ci, 3, 3, generator=g) / (ci * 9) ** 0.5) for ci, co in shapes]
    bs = [torch.randn(co, generator=g) * 0.1 for _, co in shapes]
    x = bf(torch.rand(B, 64, 16, 20, generator=g))
    conv = lambda t, k: torch.nn.functional.conv2d(t, ws[k], bs[k], padding=1)  # noqa: E731
    ref, k = bf(conv(x, 0)), 1
    for _ in range(n0 + 1 + n1):
        if k == 2 * n0 + 1:  # the widening conv (no activation, networks.py:64-72)
            ref, k = bf(conv(ref, k)), k + 1
            continue
        t = bf(torch.relu(conv(ref, k)))
        ref, k = bf(torch.relu(conv(t, k + 1) + ref)), k + 2
    return x, ws, bs, ref


@pytest.mark.parametrize("B,n0,n1", [(3, 2, 3), (5, 0, 1), (2, 1, 0), (300, 2, 3)])
def test_rep_trunk_vs_torch_fp32(B, n0, n1):
    """mzba_rep_trunk (stem, 128-channel blocks, widening conv, 256-channel blocks in one launch) against a
    plain torch fp32 evaluation of the bf16-rounded operands, every layer's output rounded to bf16: within
    2e-2 of the tensor's magnitude (test_rep_blocks_equal_band_res_launches' bound), and against the band
    launches of the same layers (the kernel sums bias and residual first, the band kernels last: most
    elements round identically)."""
    import ctypes
    from mzba import _lib as L
    from mzba.agent import pack_tower_conv, LAT_PAD_ELEMS
    x, ws, bs, ref = _trunk_case(B, n0, n1, 100 * B + 10 * n0 + n1)
    pk = lambda w: torch.from_numpy(np.concatenate([pack_tower_conv(w.numpy()),  # noqa: E731
                                                    np.zeros(LAT_PAD_ELEMS, np.float32)])).to(torch.bfloat16).cuda()
    wd = [pk(w) for w in ws]
    bd = [b.cuda() for b in bs]
    x_d = x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).cuda()
    out = torch.full((B, 16, 20, 256), float("nan"), device="cuda").to(torch.bfloat16)
    nc = len(ws)
    wp = (ctypes.c_void_p * nc)(*[t.data_ptr() for t in wd])
    bp = (ctypes.c_void_p * nc)(*[t.data_ptr() for t in bd])
    L.call("mzba_rep_trunk", L.ptr(x_d), L.ptr(out), wp, bp, n0, n1, B, L.stream())
    # the band path, layer by layer (operands held until the end): (kind, first conv index, widths)
    layers = ([("conv", 0, 64, 128)] + [("res", 1 + 2 * j, 128, 128) for j in range(n0)] +
              [("conv", 2 * n0 + 1, 128, 256)] + [("res", 2 * n0 + 2 + 2 * j, 256, 256) for j in range(n1)])
    keep, cur = [], x_d
    for kind, k, ci, co in layers:
        nxt = torch.empty(B, 16, 20, co, device="cuda", dtype=torch.bfloat16)
        if kind == "conv":
            L.call("mzba_conv_band", L.ptr(cur), L.ptr(wd[k]), L.ptr(bd[k]), None, L.ptr(nxt), B, 16, 20, ci, co, 0,
                   L.stream())
        else:
            L.call("mzba_conv_band_res", L.ptr(cur), L.ptr(wd[k]), L.ptr(bd[k]), L.ptr(wd[k + 1]), L.ptr(bd[k + 1]),
                   L.ptr(nxt), B, 16, 20, co, L.stream())
        keep.append(nxt)
        cur = nxt
    torch.cuda.synchronize()
    mag = max(1.0, ref.abs().max().item())
    got, band = out.float().cpu().permute(0, 3, 1, 2), cur.float().cpu().permute(0, 3, 1, 2)
    assert torch.isfinite(got).all()
    err, err_band = (got - ref).abs().max().item() / mag, (band - ref).abs().max().item() / mag
    same = (got == band).float().mean().item()
    print(f"rep_trunk vs torch fp32 [B={B}, n0={n0}, n1={n1}]: {err:.2e} (band: {err_band:.2e}), equal to band {same:.3f}")
    assert err < 2e-2, err
    assert err_band < 2e-2, err_band
    assert same > 0.5


@pytest.mark.parametrize("B", [13, 4096])
def test_representation_with_rep_trunk(B):
    """The whole representation net with its 16x20 trunk as one mzba_rep_trunk launch vs the band
    launches + mzba_rep_blocks, at the acting batch. The two sum bias and residual in different places
    through 16 bf16 convs, so the [0, 1] scaled root latents differ by a few bf16 steps at most (one step
    is 2^-8 .. 2^-7 on [0.5, 1]): max within 3e-2 (4 steps at 1), mean within 1e-3; the trunk is what the
    runner launches by default."""
    from mzba.agent import MuZeroAgent
    mcfg = default_config()["model"]
    ag = MuZeroAgent(mcfg, dtype="bf16")
    ag.load_state_dict(init_state_dict(mcfg, 12))
    rn = ag.runner(B, 16, 20)
    assert rn.use_rep_trunk
    g = torch.Generator().manual_seed(B + 1)
    xs = torch.rand(B, 64, 16, 20, generator=g).cuda()
    lat = {}
    for on in (True, False):
        rn.use_rep_trunk = on
        lat[on] = ag.create_hidden_state_root(xs).float().cpu()
    rn.use_rep_trunk = True
    assert torch.isfinite(lat[True]).all()
    d = (lat[True] - lat[False]).abs()
    print(f"representation, rep_trunk vs band + rep_blocks [B={B}]: max {d.max().item():.2e} mean {d.mean().item():.2e}")
    assert d.max().item() < 3e-2, d.max().item()
    assert d.mean().item() < 1e-3, d.mean().item()
