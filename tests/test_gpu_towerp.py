"""Plan 4, the pixel-tiled tower kernel (csrc/towerp.hip: 16 envs per workgroup, one MFMA tile per
latent pixel, the padding taps not issued), against plan 2 (tower8_kernel<0, 2>, column tiles of an
env quad). Every output accumulator receives the same f32 additions in the same order on both
kernels (plan 2's padded rows add exact zeros), so the outputs must be equal BIT FOR BIT: the plain
tower, the fused dynamics step (ConvBlock with the action-bias table + tower + reward head + min-max
scale, node-pool gather and write), the fused prediction step (policy / value ConvBlocks + heads) and
the prediction step's folded tree backup + selection, inside a graph-replayed 4096-env acting loop.
The parity of plan 2 itself against the reference is covered in test_gpu_parity.py."""
import numpy as np
import pytest
import torch

from mzba.config import default_config
from mzba.weights import init_state_dict

pytestmark = pytest.mark.gpu

C = 256


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"


def _plain(B, nb, variant, seed):
    from mzba import _lib as L
    g = torch.Generator().manual_seed(seed)
    S1 = 3
    x = torch.rand(B * S1 * 20 * C, generator=g).to(torch.bfloat16).cuda()
    slot = torch.randint(0, S1, (B,), generator=g, dtype=torch.int32).cuda()
    wf = (torch.randn(2 * nb * C * 2304 + 8 * 64 * 8, generator=g) * 0.02).to(torch.bfloat16).cuda()
    b = (torch.randn(2 * nb * C, generator=g) * 0.1).cuda()
    y = torch.full((B * 20 * C,), float("nan"), device="cuda").to(torch.bfloat16)
    L.call("mzba_tower_set_variant", variant)
    try:
        assert L.lib().mzba_tower_plan(B) == variant
        L.call("mzba_tower", L.ptr(x), S1 * 20 * C, L.ptr(slot), 20 * C, L.ptr(y), L.ptr(wf), L.ptr(b), nb, B, None, 0,
               L.stream())
        torch.cuda.synchronize()
    finally:
        L.call("mzba_tower_set_variant", 0)
    return y.view(torch.int16).cpu().numpy()


@pytest.mark.parametrize("B,nb", [(4096, 14), (13, 2), (40, 3)])
def test_towerp_plain_tower_bit_identical_to_tower8(B, nb):
    """mzba_tower with the slot gather: plan 4 == plan 2 bit for bit (13 / 40 envs leave the last
    16-env workgroup partly empty)."""
    a, b = _plain(B, nb, 2, B + nb), _plain(B, nb, 4, B + nb)
    assert (a != a).sum() == 0 and np.isfinite(a.view(np.uint16).astype(np.float32)).all()
    np.testing.assert_array_equal(a, b)


def _agent(seed, cfg=None, dyn_dtype=None):
    """A fresh agent per kernel: runners (and the plan each fixes at creation) are cached per batch in
    the agent's native pack."""
    from mzba.agent import MuZeroAgent
    mcfg = (cfg or default_config())["model"]
    ag = MuZeroAgent(mcfg, dtype="bf16", dyn_dtype=dyn_dtype)
    ag.load_state_dict(init_state_dict(mcfg, seed))
    return ag


def _fused(B, variant, dyn_dtype=None):
    from mzba import _lib as L
    ag = _agent(7, dyn_dtype=dyn_dtype)
    L.call("mzba_tower_set_variant", variant)
    try:
        rn = ag.runner(B, 16, 20)
    finally:
        L.call("mzba_tower_set_variant", 0)
    assert rn.fused_ok() and rn.tower_plan == variant
    S1, n = 3, 20 * C
    g = torch.Generator().manual_seed(B)
    pool = torch.rand(B, S1 + 1, n, generator=g).to(torch.bfloat16).cuda()
    slot = torch.randint(0, S1, (B,), generator=g, dtype=torch.int32).cuda()
    act = torch.randint(0, 3, (B,), generator=g, dtype=torch.int32).cuda()
    o = torch.empty(B, n, dtype=torch.bfloat16, device="cuda")
    f = lambda *s: torch.full(s, float("nan"), device="cuda")  # noqa: E731
    r, rl, pi, v, plg, vlg = f(B), f(B, 11), f(B, 3), f(B), f(B, 3), f(B, 11)
    rn.dynamics(pool, act, o, r, rl, slot=slot, env_stride=(S1 + 1) * n, slot_stride=n, pool=pool,
                pool_env_stride=(S1 + 1) * n, pool_slot=S1)
    torch.cuda.synchronize()
    r, rl = r.clone(), rl.clone()
    rn.prediction(o, pi, v, plg, vlg)
    torch.cuda.synchronize()
    out = dict(latent=o.view(torch.int16), pool=pool[:, S1].view(torch.int16), r=r.view(torch.int32),
               rl=rl.view(torch.int32), pi=pi.view(torch.int32), v=v.view(torch.int32), plg=plg.view(torch.int32),
               vlg=vlg.view(torch.int32))
    return {k: t.cpu().numpy() for k, t in out.items()}


@pytest.mark.parametrize("B", [4096, 13])
def test_towerp_fused_steps_bit_identical_to_tower8(B):
    """The fused dynamics step (prologue ConvBlock with the folded action planes, node-pool gather by
    slot, 14 blocks, reward ConvBlock 1x1 + Linear + decode, min-max scaled latent to the output and
    the pool slot) and the fused prediction step (14 blocks, policy 3x3 / value 1x1 ConvBlocks, both
    Linear heads, softmax and decode) of the random-init reference nets: plan 4 == plan 2, every output
    compared as integers."""
    a, b = _fused(B, 2), _fused(B, 4)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert np.isfinite(b["v"].view(np.float32)).all() and np.isfinite(b["pi"].view(np.float32)).all()


def test_towerp_acting_loop_bit_identical_to_tower8():
    """A graph-replayed 4096 x 50 acting loop at T < 1 (representation, 50 simulations with the tree
    backup + next selection folded into every fused prediction launch, sampling, env step, records):
    every record of 3 steps is the same on plan 4 as on plan 2."""
    from mzba import _lib as L
    from mzba.acting import ActingLoop
    cfg = default_config()
    cfg["num_simulations"] = 50
    T, B = 3, 4096

    def run(variant):
        ag = _agent(4, cfg)
        L.call("mzba_tower_set_variant", variant)
        try:
            loop = ActingLoop(cfg, ag, B, seed=29, max_steps=T, temperature=0.9)
            assert loop.ws.runner.fused_ok() and loop.ws.runner.tower_plan == variant
        finally:
            L.call("mzba_tower_set_variant", 0)
        loop.reset(0)
        loop.act(eager=True)
        loop.capture()
        for _ in range(T - 1):
            loop.act()
        torch.cuda.synchronize()
        out = {k: v[:T].cpu().numpy() for k, v in loop.rec.items() if v is not None}
        del loop, ag
        torch.cuda.empty_cache()
        return out

    a, b = run(2), run(4)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert (b["counts"].sum(-1) == 50).all()


def test_towerp_is_the_default_plan_at_16_envs_per_cu():
    """mzba_tower_plan: the pixel-tiled kernel from 16 envs per CU (the headline 4096 on 256 CUs), the
    8-env kernel from 8, the one-quad kernel below; the fp16 dynamics net falls back to the 8-env
    kernel inside mzba_tower_fused (same packing)."""
    from mzba import _lib as L
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    assert L.lib().mzba_tower_plan(16 * ncu) == 4
    assert L.lib().mzba_tower_plan(16 * ncu - 1) == 2
    assert L.lib().mzba_tower_plan(8 * ncu) == 2
    assert L.lib().mzba_tower_plan(8 * ncu - 1) == 3


@pytest.mark.parametrize("B", [4096, 13])
def test_towerp_fp16_dynamics_step_bit_identical_to_tower8(B):
    """BASELINE config 5's fp16 dynamics net (fp16 LDS image, weights and MFMAs; latents in and out
    bf16) on the pixel-tiled kernel (towerp_kernel<1>) against tower8_kernel<1, 2>: the fused dynamics
    step (and the bf16 prediction step after it) equal bit for bit."""
    a, b = _fused(B, 2, "fp16"), _fused(B, 4, "fp16")
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert np.isfinite(b["r"].view(np.float32)).all()


@pytest.mark.parametrize("B", [4096, 40])
def test_pool_only_dynamics_and_prediction_from_pool_slots(B):
    """The search's form of the fused steps: the dynamics step without `out` writes the scaled latent to
    its node-pool slot only, and the prediction step reads a [B, n] view of one slot of every env
    (env stride (S + 1) n). Against the contiguous forms (out + pool, prediction on out): every output
    equal bit for bit."""
    ag = _agent(8)
    rn = ag.runner(B, 16, 20)
    assert rn.fused_ok()
    S1, n = 3, 20 * C
    g = torch.Generator().manual_seed(B + 5)
    pool0 = torch.rand(B, S1 + 1, n, generator=g).to(torch.bfloat16).cuda()
    slot = torch.randint(0, S1, (B,), generator=g, dtype=torch.int32).cuda()
    act = torch.randint(0, 3, (B,), generator=g, dtype=torch.int32).cuda()
    res = {}
    for pool_only in (False, True):
        pool = pool0.clone()
        o = None if pool_only else torch.empty(B, n, dtype=torch.bfloat16, device="cuda")
        r = torch.full((B,), float("nan"), device="cuda")
        pi, v = torch.full((B, 3), float("nan"), device="cuda"), torch.full((B,), float("nan"), device="cuda")
        rn.dynamics(pool, act, o, r, slot=slot, env_stride=(S1 + 1) * n, slot_stride=n, pool=pool,
                    pool_env_stride=(S1 + 1) * n, pool_slot=S1)
        h = pool[:, S1] if pool_only else o
        assert h.is_contiguous() != pool_only
        rn.prediction(h, pi, v)
        torch.cuda.synchronize()
        res[pool_only] = [t.view(torch.int16 if t.dtype == torch.bfloat16 else torch.int32).cpu().numpy()
                          for t in (pool, r, pi, v)]
        if not pool_only:
            np.testing.assert_array_equal(o.view(torch.int16).cpu().numpy(), res[False][0][:, S1])
    for a, b in zip(res[False], res[True]):
        np.testing.assert_array_equal(a, b)
