"""GPU parity: the HIP path (through the C-ABI) vs the oracle / golden fixtures.
Run on the MI355X box: python -m pytest tests -m gpu -x -q"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import rng as R
from oracle.env import BreakoutEnvOracle, convert_to_grayscale
from oracle import nets as N
from oracle.mcts import MCTSOracle, NetModel
from oracle.acting import prepare_mcts_input, sample_actions, run_episode, Trajectory
from mzba.config import default_config, small_model_cfg
from mzba.weights import init_state_dict

pytestmark = pytest.mark.gpu

ENV_CFG = default_config()["environment"]


def unpack(p, H, W):
    B = p.shape[0]
    return np.unpackbits(p, axis=-1)[..., : H * W].reshape(B, 3, H, W).astype(np.float32)


def dev(x, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(x), device="cuda")
    return t.to(dtype) if dtype is not None else t


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    from mzba import _lib
    _lib.lib()


# ------------------------------------------------------------------------------ env
@pytest.mark.parametrize("tag", ["16x20", "84x84"])
def test_env_planes_trajectory(tag):
    from mzba.env import BreakoutEnvironment
    d = np.load(os.path.join(GOLDEN, f"env_{tag}.npz"))
    B, H, W, seed = int(d["B"]), int(d["H"]), int(d["W"]), int(d["seed"])
    e = BreakoutEnvironment({**ENV_CFG, "n_parallel": B}, seed=seed)
    e.height, e.width = H, W
    s, _ = e.reset()  # device Philox draws == oracle reset_params == reference (fixture)
    np.testing.assert_array_equal(s.cpu().numpy(), unpack(d["states"][0], H, W))
    np.testing.assert_array_equal(e.ball_dx.cpu().numpy(), d["dx"][0])
    done = torch.zeros(B, dtype=torch.bool, device="cuda")
    for t in range(d["actions"].shape[0]):
        s, r, done2, v = e.step(s, dev(d["actions"][t]), done)
        assert done2 is done
        np.testing.assert_array_equal(s.cpu().numpy(), unpack(d["states"][t + 1], H, W), err_msg=f"t={t}")
        np.testing.assert_array_equal(r.cpu().numpy(), d["rewards"][t])
        np.testing.assert_array_equal(done.cpu().numpy(), d["dones"][t])
        np.testing.assert_array_equal(v.cpu().numpy(), d["valids"][t])
        np.testing.assert_array_equal(e.ball_dx.cpu().numpy(), d["dx"][t + 1])
        np.testing.assert_array_equal(e.ball_dy.cpu().numpy(), d["dy"][t + 1])


def test_torch_op_env_step_matches_reference():
    """torch.ops.mz.env_reset_ / env_step / grayscale (TORCH_LIBRARY(mz), csrc/torch_ops.cpp) on the
    reference's 16x20 trajectory: done is mutated in place and returned as the same tensor
    (schema Tensor(a!) done -> Tensor(a!)), every output bit-exact."""
    from mzba import _lib as L
    ops = L.ops()
    d = np.load(os.path.join(GOLDEN, "env_16x20.npz"))
    B, H, W, seed = int(d["B"]), int(d["H"]), int(d["W"]), int(d["seed"])
    s = torch.empty(B, 3, H, W, device="cuda")
    dx = torch.empty(B, dtype=torch.int64, device="cuda")
    dy = torch.empty(B, dtype=torch.float32, device="cuda")
    ops.env_reset_(s, dx, dy, 6, 3, seed, 0, 0, None)
    np.testing.assert_array_equal(s.cpu().numpy(), unpack(d["states"][0], H, W))
    done = torch.zeros(B, dtype=torch.bool, device="cuda")
    r4 = [float(ENV_CFG[k]) for k in ("paddle_hit_reward", "brick_hit_reward", "game_lost_reward", "game_won_reward")]
    for t in range(d["actions"].shape[0]):
        s, r, d2, v, dx, dy = ops.env_step(s, dev(d["actions"][t]), done, dx, dy, 6, r4)
        assert d2 is done or d2.data_ptr() == done.data_ptr()
        np.testing.assert_array_equal(s.cpu().numpy(), unpack(d["states"][t + 1], H, W), err_msg=f"t={t}")
        np.testing.assert_array_equal(r.cpu().numpy(), d["rewards"][t])
        np.testing.assert_array_equal(done.cpu().numpy(), d["dones"][t])
        np.testing.assert_array_equal(v.cpu().numpy(), d["valids"][t])
        np.testing.assert_array_equal(dx.cpu().numpy(), d["dx"][t + 1])
        np.testing.assert_array_equal(dy.cpu().numpy(), d["dy"][t + 1])
    np.testing.assert_array_equal(ops.grayscale(s).cpu().numpy(), convert_to_grayscale(s.cpu().numpy()))
    with pytest.raises(RuntimeError):  # TORCH_CHECK on a malformed call
        ops.env_step(s, dev(d["actions"][0][:3]), done, dx, dy, 6, r4)


@pytest.mark.parametrize("tag", ["16x20", "84x84"])
def test_env_planes_fuzz(tag):
    from mzba.env import BreakoutEnvironment
    d = np.load(os.path.join(GOLDEN, f"envfuzz_{tag}.npz"))
    B, H, W = int(d["B"]), int(d["H"]), int(d["W"])
    e = BreakoutEnvironment({**ENV_CFG, "n_parallel": B})
    e.height, e.width = H, W
    e.ball_dx, e.ball_dy = dev(d["dx"]), dev(d["dy"])
    done = dev(d["done"])
    ns, r, dn, v = e.step(dev(unpack(d["state"], H, W)), dev(d["action"]), done)
    np.testing.assert_array_equal(ns.cpu().numpy(), unpack(d["next_state"], H, W))
    np.testing.assert_array_equal(r.cpu().numpy(), d["reward"])
    np.testing.assert_array_equal(dn.cpu().numpy(), d["next_done"])
    np.testing.assert_array_equal(v.cpu().numpy(), d["valid"])
    np.testing.assert_array_equal(e.ball_dx.cpu().numpy(), d["next_dx"])
    np.testing.assert_array_equal(e.ball_dy.cpu().numpy(), d["next_dy"])


def test_env_planes_cpu_tensors_roundtrip():
    """Drop-in: CPU state/done tensors in, CPU out, done mutated in place."""
    from mzba.env import BreakoutEnvironment
    e = BreakoutEnvironment({**ENV_CFG, "n_parallel": 8}, seed=3)
    s, _ = e.reset()
    s = s.cpu()
    done = torch.zeros(8, dtype=torch.bool)
    for t in range(40):
        ns, r, d2, v = e.step(s, torch.full((8,), t % 3), done)
        assert d2 is done and ns.device.type == "cpu"
        s = ns


def test_env_bad_state_raises():
    from mzba.env import BreakoutEnvironment
    e = BreakoutEnvironment({**ENV_CFG, "n_parallel": 2})
    s, _ = e.reset()
    s[:, 1] = 0  # no ball
    with pytest.raises(IndexError):
        e.step(s, torch.zeros(2, dtype=torch.int64, device="cuda"), torch.zeros(2, dtype=torch.bool, device="cuda"))


@pytest.mark.parametrize("tag", ["16x20", "84x84"])
def test_env_compact_matches_planes_and_reference(tag):
    from mzba.env import CompactBreakout
    d = np.load(os.path.join(GOLDEN, f"env_{tag}.npz"))
    B, H, W, seed = int(d["B"]), int(d["H"]), int(d["W"]), int(d["seed"])
    env = CompactBreakout(ENV_CFG, B, 4, H, W, seed=seed)
    env.reset(0)
    np.testing.assert_array_equal(env.to_planes().cpu().numpy(), unpack(d["states"][0], H, W))
    from mzba.env import gray_lut
    lut = gray_lut()
    for t in range(d["actions"].shape[0]):
        env.step(dev(d["actions"][t]), t == 0)
        ref = unpack(d["states"][t + 1], H, W)
        np.testing.assert_array_equal(env.to_planes().cpu().numpy(), ref, err_msg=f"t={t}")
        np.testing.assert_array_equal(env.reward.cpu().numpy(), d["rewards"][t])
        np.testing.assert_array_equal(env.done.cpu().numpy().astype(bool), d["dones"][t])
        np.testing.assert_array_equal(env.valid.cpu().numpy(), d["valids"][t])
        g = lut[env.current_frame().view(B, H * W).cpu().numpy() & 7].reshape(B, 1, H, W)
        np.testing.assert_array_equal(g, convert_to_grayscale(ref))


def test_grayscale_kernel():
    from mzba.env import grayscale
    g = np.random.default_rng(0)
    s = (g.random((64, 3, 16, 20)) < 0.3).astype(np.float32)
    np.testing.assert_array_equal(grayscale(dev(s)).cpu().numpy(), convert_to_grayscale(s))


def _oracle_history(B, L, H, W, steps, seed):
    """Oracle env + trajectories for `steps` random actions (record rule of :204-209)."""
    e = BreakoutEnvOracle({**ENV_CFG, "n_parallel": B})
    e.height, e.width = H, W
    s, _ = e.reset(e.reset_params(seed, 0))
    g0 = convert_to_grayscale(s)
    trajs = [Trajectory(L, g0[b]) for b in range(B)]
    done = np.zeros(B, bool)
    prev = done
    acts = []
    for t in range(steps):
        a = R.randbelow(np.arange(B), 9, t, 0, seed, 3)
        acts.append(a)
        s, r, done, v = e.step(s, a, done)
        w = convert_to_grayscale(s)
        for b in range(B):
            if not prev[b]:
                trajs[b].add_observation(a[b], w[b], r[b], np.zeros(3, np.int64), 0.0)
        prev = done.copy()
    return trajs, convert_to_grayscale(s), acts


@pytest.mark.parametrize("single_write", [True, False])
@pytest.mark.parametrize("L,steps", [(32, 0), (32, 5), (32, 45), (4, 7), (4, 120)])
def test_rep_input_builder(L, steps, single_write):
    """single_write: recorded frames only in the ring (cur_src) vs also copied to cur_frame;
    (4, 120) leaves most envs done, so both frame locations are read."""
    from mzba.env import CompactBreakout, gray_lut
    B, H, W, seed = 16, 16, 20, 11
    trajs, cur, acts = _oracle_history(B, L, H, W, steps, seed)
    env = CompactBreakout(ENV_CFG, B, L, H, W, seed=seed, single_write=single_write)
    env.reset(0)
    for t in range(steps):
        env.step(dev(acts[t]), t == 0)
    cs = (2 * L + 63) // 64 * 64
    out = torch.empty(B * H * W * cs, dtype=torch.float32, device="cuda")
    env.build_rep_input(out, cs, False)
    got = out.view(B, H, W, cs).permute(0, 3, 1, 2).cpu().numpy()
    ref = np.stack([prepare_mcts_input(cur[b], trajs[b], L) for b in range(B)])
    np.testing.assert_array_equal(got[:, : 2 * L], ref)
    assert not got[:, 2 * L:].any()
    lut = gray_lut()
    np.testing.assert_array_equal(lut[env.current_frame().view(B, H, W).cpu().numpy() & 7], cur[:, 0])
    if single_write and steps in (5, 120):  # both frame locations exercised
        src = env.cur_src.cpu().numpy()
        assert (src == 1).all() if steps == 5 else (src == 0).all(), src


# ------------------------------------------------------------------------------ nets
@pytest.mark.parametrize("tag,x6,x3", [("small", 2, 0), ("full", 2, 0), ("full", 3, 0), ("full", 2, 1)])
def test_nets_f32_match_reference(tag, x6, x3):
    """The f32 parity path's nets on the reference's own outputs (nets_*.npz) within 1e-5. x6 = 3: every 4x5 latent
    3x3 conv on the pixel-tiled x6 form (the form the 4096-env parity path runs: the towers, the dynamics' first
    conv with its gather + action bias, the policy head's conv); 2: the form chosen by batch (pre-split here).
    x3 = 1 (round 6): the 4x5 latent's convs on the split-fp16 x3 form instead (mzba_conv_x3_ex), the same 1e-5."""
    from mzba import _lib as L
    from mzba.agent import MuZeroAgent
    d = np.load(os.path.join(GOLDEN, f"nets_{tag}.npz"))
    cfg = default_config()
    mcfg = cfg["model"] if tag == "full" else small_model_cfg(cfg)
    ag = MuZeroAgent(mcfg, dtype="f32")
    ag.load_state_dict(init_state_dict(mcfg, int(d["weight_seed"])))
    ag.packed.native.set_int("use_x3", x3)  # before the first op creates this batch's runner
    tol = dict(rtol=1e-5, atol=1e-5)  # north_star: within 1e-5 for network logits/values
    try:
        assert L.lib().mzba_conv_x6_set_variant(x6) == 0
        h = ag.create_hidden_state_root(dev(d["x"])).cpu().numpy()
        np.testing.assert_allclose(h, d["h"], **tol)
        pl, vl = ag.evaluate_state(dev(d["h"]))
        np.testing.assert_allclose(pl.cpu().numpy(), d["p0"], **tol)
        np.testing.assert_allclose(vl.cpu().numpy(), d["v0"], **tol)
        planes = N.encode_action_planes(d["action"], mcfg["latent_resolution"])
        h1, rl = ag.hidden_state_transition(dev(d["h"]), dev(planes))
        np.testing.assert_allclose(h1.cpu().numpy(), d["h1"], **tol)
        np.testing.assert_allclose(rl.cpu().numpy(), d["r1"], **tol)
    finally:
        L.lib().mzba_conv_x6_set_variant(2)
    if tag == "full":  # the 4x5 latent's 3x3 convs all carry x6 weights (round 5: dyn0 and the policy conv too)
        p = ag.packed    # and x3 weights (round 6)
        assert p.dyn0.get("wx") is not None and p.pol_conv.get("wx") is not None
        assert all(c.get("wx") is not None and c.get("wx3") is not None for blk in p.dyn + p.pred for c in blk)
        assert p.dyn0.get("wx3") is not None and p.pol_conv.get("wx3") is not None


def test_nets_bf16_close():
    from mzba.agent import MuZeroAgent
    d = np.load(os.path.join(GOLDEN, "nets_full.npz"))
    mcfg = default_config()["model"]
    ag = MuZeroAgent(mcfg, dtype="bf16")
    ag.load_state_dict(init_state_dict(mcfg, int(d["weight_seed"])))
    h = ag.create_hidden_state_root(dev(d["x"])).cpu().numpy()
    assert np.abs(h - d["h"]).max() < 0.05
    pl, vl = ag.evaluate_state(dev(d["h"]))
    assert np.abs(pl.cpu().numpy() - d["p0"]).max() < 0.05
    assert np.abs(vl.cpu().numpy() - d["v0"]).max() < 0.05
    planes = N.encode_action_planes(d["action"], mcfg["latent_resolution"])
    h1, rl = ag.hidden_state_transition(dev(d["h"]), dev(planes))
    assert np.abs(h1.cpu().numpy() - d["h1"]).max() < 0.05
    assert np.abs(rl.cpu().numpy() - d["r1"]).max() < 0.05


@pytest.mark.parametrize("B,variant", [(13, 1), (1024, 1), (13, 2), (2048, 0), (13, 3), (1024, 3), (13, 4), (40, 4)])
def test_fused_steps_match_unfused(B, variant):
    """mzba_tower_fused (dynamics ConvBlock + tower + reward head + scale in one launch; tower +
    policy/value heads in one launch) vs the per-layer launch sequence, both bf16, same inputs;
    on the 4-env (variant 1) and the 8-env kernel (2; 0 = by batch: 2048 plans the 8-env one)."""
    from mzba import _lib as L
    from mzba.agent import MuZeroAgent
    mcfg = default_config()["model"]
    ag = MuZeroAgent(mcfg, dtype="bf16")
    ag.load_state_dict(init_state_dict(mcfg, 7))
    L.call("mzba_tower_set_variant", variant)
    try:
        rn = ag.runner(B, 16, 20)
    finally:
        L.call("mzba_tower_set_variant", 0)
    assert rn.fused_ok() and rn.tower_plan == (variant or 2)
    S1, n = 3, 20 * 256
    g = torch.Generator().manual_seed(B)
    pool0 = torch.rand(B, S1 + 1, n, generator=g).to(torch.bfloat16).cuda()
    slot = torch.randint(0, S1, (B,), generator=g, dtype=torch.int32).cuda()
    act = torch.randint(0, 3, (B,), generator=g, dtype=torch.int32).cuda()
    res = {}
    try:
        for fused in (False, True):
            rn.use_fused = fused
            pool = pool0.clone()
            out = torch.empty(B, n, dtype=torch.bfloat16, device="cuda")
            f = lambda *s: torch.full(s, float("nan"), device="cuda")  # noqa: E731
            r, rl, pi, v, plg, vlg = f(B), f(B, 11), f(B, 3), f(B), f(B, 3), f(B, 11)
            rn.dynamics(pool, act, out, r, rl, slot=slot, env_stride=(S1 + 1) * n, slot_stride=n, pool=pool,
                        pool_env_stride=(S1 + 1) * n, pool_slot=S1)
            rn.prediction(out, pi, v, plg, vlg)
            torch.cuda.synchronize()
            res[fused] = [t.float().cpu() for t in (out, pool[:, S1], r, rl, pi, v, plg, vlg)]
    finally:
        rn.use_fused = True
    names = ["latent", "pool", "r", "r_logits", "pi", "v", "p_logits", "v_logits"]
    for nm, a, b in zip(names, res[False], res[True]):
        assert torch.isfinite(b).all(), nm
        err = (a - b).abs().max().item()
        assert err < 0.05, (nm, err)
    assert torch.equal(res[True][0], res[True][1])  # scaled latent also written to the pool slot


def _bf(t):
    return t.to(torch.bfloat16).float()


class _Bf16StepRef:
    """Plain torch fp32 reference of the fused bf16 dynamics / prediction steps (CPU), rounding to
    bf16 exactly where the kernels store bf16: BN folded in f64 (networks.py:7-35 eval) then weights
    rounded f64 -> f32 -> bf16, every ReLU output (the LDS images) rounded to bf16, f32 everywhere
    else (accumulators, biases, the action-plane bias table, Linear heads, min-max scale)."""

    def __init__(self, sd, mcfg):
        self.sd = {k: np.asarray(v, np.float64) for k, v in sd.items()}
        self.c1 = mcfg["latent_channels"][1]
        self.nd = mcfg["dynamics_network"]["num_res_blocks"]
        self.np_ = mcfg["prediction_network"]["num_res_blocks"]

    def _fold(self, p, bn):
        s = self.sd
        a = s[bn + ".weight"] / np.sqrt(s[bn + ".running_var"] + 1e-5)
        w = s[p + ".weight"] * a[:, None, None, None]
        b = s[p + ".bias"] * a + (s[bn + ".bias"] - s[bn + ".running_mean"] * a)
        return torch.tensor(w, dtype=torch.float32), torch.tensor(b, dtype=torch.float32)

    def _conv(self, x, p, bn, pad, extra=None):
        w, b = self._fold(p, bn)
        y = torch.nn.functional.conv2d(x, _bf(w[:, : x.shape[1]]), b, padding=pad)
        return y if extra is None else y + extra

    def _lin(self, x, p):
        return torch.nn.functional.linear(x.flatten(1), _bf(torch.tensor(self.sd[p + ".weight"], dtype=torch.float32)),
                                          torch.tensor(self.sd[p + ".bias"], dtype=torch.float32))

    def _tower(self, x, prefix, n):
        for i in range(n):
            p = f"{prefix}.{i}"
            t = _bf(torch.relu(self._conv(x, p + ".conv1", p + ".bn1", 1)))
            x = _bf(torch.relu(self._conv(t, p + ".conv2", p + ".bn2", 1, extra=x)))
        return x

    def dynamics(self, h, act):
        """h: bf16-valued f32 NCHW latent, act: i64[B] -> scaled latent (bf16 values), reward logits."""
        w, _ = self._fold("dyn_net.conv_block.conv", "dyn_net.conv_block.bn")
        planes = torch.nn.functional.one_hot(act, 3).float()[:, :, None, None].expand(-1, -1, *h.shape[2:])
        # the 3 action channels stay f32 (the kernels' per-(pixel, action) bias table)
        ab = torch.nn.functional.conv2d(planes, w[:, self.c1:], None, padding=1)
        x = _bf(torch.relu(self._conv(h, "dyn_net.conv_block.conv", "dyn_net.conv_block.bn", 1, extra=ab)))
        x = self._tower(x, "dyn_net.res_blocks", self.nd)
        r = _bf(torch.relu(self._conv(x, "dyn_net.reward_head.0.conv", "dyn_net.reward_head.0.bn", 0)))
        rl = self._lin(r, "dyn_net.reward_head.2")
        f = x.flatten(1)
        mn, mx = f.min(1).values[:, None, None, None], f.max(1).values[:, None, None, None]
        return _bf((x - mn) / ((mx - mn) + 1e-8)), rl

    def prediction(self, h):
        x = self._tower(h, "pred_net.res_blocks", self.np_)
        p = _bf(torch.relu(self._conv(x, "pred_net.policy_head.0.conv", "pred_net.policy_head.0.bn", 1)))
        v = _bf(torch.relu(self._conv(x, "pred_net.value_head.0.conv", "pred_net.value_head.0.bn", 0)))
        return self._lin(p, "pred_net.policy_head.2"), self._lin(v, "pred_net.value_head.2")


@pytest.mark.parametrize("B,variant", [(13, 1), (64, 2), (13, 3), (64, 0), (13, 4), (64, 4)])
def test_fused_bf16_steps_vs_torch_fp32(B, variant):
    """The fused bf16 dynamics and prediction launches (ConvBlock + 14 residual blocks + heads +
    min-max scale in one launch each) against a plain torch fp32 evaluation of the same folded,
    bf16-rounded weights with bf16 activations where the kernels keep bf16 (_Bf16StepRef). The
    remaining differences are f32 summation order inside a conv, each worth at most one bf16 ulp
    of an activation; the tolerance, 2e-2 of the tensor's magnitude for the scaled latent and the
    logits, is the one test_tower_matches_conv_chain uses for the plain tower."""
    from mzba import _lib as L
    from mzba.agent import MuZeroAgent
    mcfg = default_config()["model"]
    sd = init_state_dict(mcfg, 7)
    ag = MuZeroAgent(mcfg, dtype="bf16")
    ag.load_state_dict(sd)
    L.call("mzba_tower_set_variant", variant)
    try:
        rn = ag.runner(B, 16, 20)
    finally:
        L.call("mzba_tower_set_variant", 0)
    assert rn.fused_ok() and rn.tower_plan == (variant or L.lib().mzba_tower_plan(B))
    n = 20 * 256
    g = torch.Generator().manual_seed(B + variant)
    src = torch.rand(B, n, generator=g).to(torch.bfloat16)
    act = torch.randint(0, 3, (B,), generator=g)
    lat = torch.empty(B, n, dtype=torch.bfloat16, device="cuda")
    f = lambda *s: torch.full(s, float("nan"), device="cuda")  # noqa: E731
    r, rl, pi, v, plg, vlg = f(B), f(B, 11), f(B, 3), f(B), f(B, 3), f(B, 11)
    rn.dynamics(src.cuda(), act.to(torch.int32).cuda(), lat, r, rl)
    rn.prediction(lat, pi, v, plg, vlg)
    torch.cuda.synchronize()
    ref = _Bf16StepRef(sd, mcfg)
    nchw = lambda t: t.float().cpu().view(B, 4, 5, 256).permute(0, 3, 1, 2)  # noqa: E731
    h_ref, rl_ref = ref.dynamics(nchw(src), act)
    pl_ref, vl_ref = ref.prediction(nchw(lat))  # the kernel's own latent: isolates the prediction step
    for nm, got, want in (("latent", nchw(lat), h_ref), ("reward_logits", rl.cpu(), rl_ref),
                          ("policy_logits", plg.cpu(), pl_ref), ("value_logits", vlg.cpu(), vl_ref)):
        assert torch.isfinite(got).all(), nm
        err = (got - want).abs().max().item() / max(1.0, want.abs().max().item())
        print(f"bf16 fused step vs torch fp32 [B={B}, variant={variant}] {nm}: {err:.2e}")
        assert err < 2e-2, (nm, err)


@pytest.mark.parametrize("B", [1, 13, 256])
def test_rep_tail_vs_torch_fp32(B):
    """mzba_rep_tail (AvgPool2d 16x20 -> 8x10, the 3 ResidualBlock(256) at 8x10, AvgPool2d -> 4x5 and
    _scale_state in one launch, networks.py:86-99, 314-328) against a plain torch fp32 evaluation with
    bf16 rounding where the unfused launch sequence stores bf16 (pooled maps, ReLU outputs, scaled
    latent); and the whole representation net with the fused tail against the unfused launches.
    Tolerance 2e-2 absolute on the [0, 1] scaled latent (f32 summation order inside the convs); odd B
    leaves the last workgroup one env short."""
    from mzba import _lib as L
    from mzba.agent import MuZeroAgent
    from mzba.weights import rep_layout
    mcfg = default_config()["model"]
    sd = init_state_dict(mcfg, 11)
    ag = MuZeroAgent(mcfg, dtype="bf16")
    ag.load_state_dict(sd)
    tail = ag.packed.rep_tail
    assert tail is not None and tail["n"] == 3
    g = torch.Generator().manual_seed(B)
    x = torch.rand(B, 320, 256, generator=g).to(torch.bfloat16)
    out = torch.full((B, 20, 256), float("nan"), device="cuda").to(torch.bfloat16)
    pool = torch.zeros(B, 3, 20, 256, device="cuda").to(torch.bfloat16)
    L.call("mzba_rep_tail", L.ptr(x.cuda()), L.ptr(out), L.ptr(pool), 3 * 20 * 256, L.ptr(tail["wf"]), L.ptr(tail["b"]),
           3, B, L.stream())
    torch.cuda.synchronize()
    ref = _Bf16StepRef(sd, mcfg)
    lay = rep_layout(mcfg)
    h = x.float().view(B, 16, 20, 256).permute(0, 3, 1, 2)
    pool2 = lambda t: _bf((((t[:, :, 0::2, 0::2] + t[:, :, 0::2, 1::2]) + t[:, :, 1::2, 0::2]) + t[:, :, 1::2, 1::2]) / 4.0)  # noqa: E731
    h = pool2(h)
    for j in [i for k, i in lay[tail["first"] + 1: -1]]:
        p = f"rep_net.blocks.{j}"
        t = _bf(torch.relu(ref._conv(h, p + ".conv1", p + ".bn1", 1)))
        h = _bf(torch.relu(ref._conv(t, p + ".conv2", p + ".bn2", 1, extra=h)))
    h = pool2(h)
    f = h.flatten(1)
    mn, mx = f.min(1).values[:, None, None, None], f.max(1).values[:, None, None, None]
    want = _bf((h - mn) / ((mx - mn) + 1e-8))
    got = out.float().cpu().view(B, 4, 5, 256).permute(0, 3, 1, 2)
    assert torch.isfinite(got).all()
    err = (got - want).abs().max().item()
    print(f"rep tail vs torch fp32 [B={B}]: {err:.2e}")
    assert err < 2e-2, err
    assert torch.equal(pool[:, 0].cpu(), out.cpu())  # slot 0 of the node pool = the root latent
    # the whole representation net, fused tail vs the unfused launches (same bf16 weights)
    xs = torch.rand(B, 64, 16, 20, generator=g).cuda()
    rn = ag.runner(B, 16, 20)
    lat = {}
    for fused in (True, False):
        rn.use_rep_tail = fused
        lat[fused] = ag.create_hidden_state_root(xs).float().cpu()
    rn.use_rep_tail = True
    d = (lat[True] - lat[False]).abs().max().item()
    print(f"representation, fused tail vs unfused [B={B}]: {d:.2e}")
    assert d < 2e-2, d


@pytest.mark.parametrize("Cin,Cout,resid,relu", [(64, 128, False, False), (128, 128, False, True), (128, 256, False, False),
                                                   (256, 256, True, True), (256, 128, False, True)])
@pytest.mark.parametrize("xt", [10, 5])
def test_band_conv_vs_torch_fp32(Cin, Cout, resid, relu, xt):
    """16x20 band kernel (10- and 5-column bands) vs a plain torch fp32 conv (bf16-rounded operands),
    incl. residual + ReLU."""
    from mzba import _lib as L
    from mzba.agent import pack_tower_conv, LAT_PAD_ELEMS
    B, H, W = 5, 16, 20
    g = torch.Generator().manual_seed(Cin + Cout)
    bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    x = bf(torch.randn(B, Cin, H, W, generator=g))
    w = bf(torch.randn(Cout, Cin, 3, 3, generator=g) / (Cin * 9) ** 0.5)
    b = torch.randn(Cout, generator=g)
    res = bf(torch.randn(B, Cout, H, W, generator=g))
    ref = torch.nn.functional.conv2d(x, w, b, padding=1) + (res if resid else 0)
    ref = torch.relu(ref) if relu else ref
    d = dict(x=x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).cuda(),
             w=torch.from_numpy(np.concatenate([pack_tower_conv(w.numpy()), np.zeros(LAT_PAD_ELEMS, np.float32)]))
             .to(torch.bfloat16).cuda(), b=b.cuda(), r=res.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).cuda())
    out = torch.empty(B, H, W, Cout, dtype=torch.bfloat16, device="cuda")
    assert L.lib().mzba_conv_band_supported(H, W, Cin, Cout, 3)
    L.call("mzba_conv_band_set_xt", xt)
    try:
        L.call("mzba_conv_band", L.ptr(d["x"]), L.ptr(d["w"]), L.ptr(d["b"]), L.ptr(d["r"]) if resid else None,
               L.ptr(out), B, H, W, Cin, Cout, 1 if relu else 0, L.stream())
    finally:
        L.call("mzba_conv_band_set_xt", 5)
    got = out.float().cpu().permute(0, 3, 1, 2)
    err = (got - ref).abs().max().item() / max(1.0, ref.abs().max().item())
    assert err < 1e-2, err


@pytest.mark.parametrize("C,B", [(256, 5), (128, 3), (256, 130)])
def test_band_res_block_equals_two_band_convs(C, B):
    """mzba_conv_band_res (a representation ResidualBlock at 16x20 in one launch: the 10-column band
    LDS-resident across both convs, conv1 recomputing one halo column each side) against the two
    mzba_conv_band launches it replaces, bit for bit (same k loop, same bf16 store of conv1's output),
    and against a plain torch fp32 block of the bf16-rounded operands; and the representation net
    with the fused blocks against the per-conv launches, bit for bit."""
    from mzba import _lib as L
    from mzba.agent import MuZeroAgent, pack_tower_conv, LAT_PAD_ELEMS
    g = torch.Generator().manual_seed(C + B)
    bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    x = bf(torch.rand(B, C, 16, 20, generator=g))
    w1, w2 = (bf(torch.randn(C, C, 3, 3, generator=g) / (C * 9) ** 0.5) for _ in range(2))
    b1, b2 = torch.randn(C, generator=g) * 0.1, torch.randn(C, generator=g) * 0.1
    pk = lambda w: torch.from_numpy(np.concatenate([pack_tower_conv(w.numpy()), np.zeros(LAT_PAD_ELEMS, np.float32)])).to(torch.bfloat16).cuda()  # noqa: E731
    d = dict(x=x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).cuda(), w1=pk(w1), w2=pk(w2), b1=b1.cuda(),
             b2=b2.cuda())
    t = torch.empty(B, 16, 20, C, dtype=torch.bfloat16, device="cuda")
    two = torch.empty_like(t)
    one = torch.full_like(t, float("nan"))
    assert L.lib().mzba_conv_band_res_supported(16, 20, C)
    L.call("mzba_conv_band", L.ptr(d["x"]), L.ptr(d["w1"]), L.ptr(d["b1"]), None, L.ptr(t), B, 16, 20, C, C, 1, L.stream())
    L.call("mzba_conv_band", L.ptr(t), L.ptr(d["w2"]), L.ptr(d["b2"]), L.ptr(d["x"]), L.ptr(two), B, 16, 20, C, C, 1,
           L.stream())
    L.call("mzba_conv_band_res", L.ptr(d["x"]), L.ptr(d["w1"]), L.ptr(d["b1"]), L.ptr(d["w2"]), L.ptr(d["b2"]),
           L.ptr(one), B, 16, 20, C, L.stream())
    torch.cuda.synchronize()
    assert torch.equal(one, two)
    ref = torch.relu(torch.nn.functional.conv2d(bf(torch.relu(torch.nn.functional.conv2d(x, w1, b1, padding=1))), w2, b2,
                                                padding=1) + x)
    err = (one.float().cpu().permute(0, 3, 1, 2) - ref).abs().max().item() / max(1.0, ref.abs().max().item())
    assert err < 2e-2, err
    if C == 256 and B == 5:  # the whole representation net: fused blocks == per-conv launches
        mcfg = default_config()["model"]
        ag = MuZeroAgent(mcfg, dtype="bf16")
        ag.load_state_dict(init_state_dict(mcfg, 12))
        rn = ag.runner(B, 16, 20)
        xs = torch.rand(B, 64, 16, 20, generator=g).cuda()
        lat = {}
        for fused in (True, False):
            rn.use_band_res = fused
            lat[fused] = ag.create_hidden_state_root(xs).cpu()
        rn.use_band_res = True
        assert torch.equal(lat[True], lat[False])


def test_conv_kernel_vs_torch_fp32_random():
    """Raw conv op vs a plain torch fp32 conv, ragged M (B*HW not a tile multiple), 1x1 and 3x3."""
    from mzba import _lib as L
    g = torch.Generator().manual_seed(0)
    for (B, H, W, Cin, Cout, ks) in [(3, 4, 5, 64, 96, 3), (7, 16, 20, 64, 128, 3), (5, 4, 5, 256, 256, 1),
                                     (2, 8, 10, 128, 32, 3)]:
        x = torch.randn(B, Cin, H, W, generator=g)
        w = torch.randn(Cout, Cin, ks, ks, generator=g) / (Cin * ks * ks) ** 0.5
        b = torch.randn(Cout, generator=g)
        res = torch.randn(B, Cout, H, W, generator=g)
        ref = torch.relu(torch.nn.functional.conv2d(x, w, b, padding=ks // 2) + res)
        for dt, tol in ((0, 2e-5), (1, 6e-2)):
            tdt = torch.float32 if dt == 0 else torch.bfloat16
            xd = x.permute(0, 2, 3, 1).contiguous().to(tdt).cuda()
            wd = w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous().to(tdt).cuda()
            rd = res.permute(0, 2, 3, 1).contiguous().to(tdt).cuda()
            out = torch.empty(B, H, W, Cout, dtype=tdt, device="cuda")
            bd = b.cuda()
            L.call("mzba_conv2d", dt, L.ptr(xd), H * W * Cin, None, 0, L.ptr(wd), L.ptr(bd), None, None, 0,
                   L.ptr(rd), L.ptr(out), B, H, W, Cin, Cout, ks, 1, L.stream())
            got = out.float().permute(0, 3, 1, 2).cpu()
            err = (got - ref).abs().max().item() / max(1.0, ref.abs().max().item())
            assert err < tol, (B, H, W, Cin, Cout, ks, dt, err)


@pytest.mark.parametrize("B,H,W,Cin,Cout,ks,relu", [(150, 21, 21, 256, 256, 3, 1), (12, 84, 84, 128, 256, 3, 0),
                                                     (40, 42, 42, 256, 256, 1, 1), (130, 21, 21, 64, 512, 3, 1)])
def test_conv_big_kernel_vs_torch_fp32(B, H, W, Cin, Cout, ks, relu):
    """The 256 x 256 large-image bf16 conv (mzba_conv2d on >= 64K pixels: config 3's 84x84 / 42x42
    images and 21x21 latents) vs a torch fp32 conv of the same bf16 operands (+ bias, residual,
    ReLU), ragged pixel counts; and close to the generic kernel (variant 0)."""
    from mzba import _lib as L
    g = torch.Generator(device="cuda").manual_seed(B + Cin)
    dev = torch.device("cuda")
    x = torch.randn(B, H, W, Cin, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(Cout, ks, ks, Cin, generator=g, device=dev) / (Cin * ks * ks) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, generator=g, device=dev)
    res = torch.randn(B, H, W, Cout, generator=g, device=dev).to(torch.bfloat16)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=ks // 2)
    ref = ref.permute(0, 2, 3, 1) + res.float()
    if relu:
        ref = torch.relu(ref)
    outs = []
    for variant in (1, 0):
        out = torch.empty(B, H, W, Cout, dtype=torch.bfloat16, device=dev)
        L.call("mzba_conv2d_set_variant", variant)
        try:
            L.call("mzba_conv2d", 1, L.ptr(x), H * W * Cin, None, 0, L.ptr(w), L.ptr(b), None, None, 0, L.ptr(res),
                   L.ptr(out), B, H, W, Cin, Cout, ks, relu, L.stream())
        finally:
            L.call("mzba_conv2d_set_variant", 1)
        outs.append(out.float())
    scale = ref.abs().max().item()
    assert (outs[0] - ref).abs().max().item() <= 1e-2 * scale  # bf16 output rounding
    assert (outs[0] - outs[1]).abs().max().item() <= 1e-2 * scale


@pytest.mark.parametrize("B,H,W,Cin,Cout,relu,with_res", [(150, 21, 21, 256, 256, 1, True), (37, 21, 21, 256, 256, 0, False),
                                                          (12, 84, 84, 128, 256, 0, True), (9, 16, 20, 256, 256, 1, True),
                                                          (3, 21, 21, 256, 512, 1, True), (37, 21, 21, 256, 128, 1, False),
                                                          (20, 21, 21, 256, 128, 0, True), (5, 84, 84, 256, 256, 1, True),
                                                          (9, 42, 42, 256, 256, 0, False), (6, 84, 84, 128, 128, 1, True)])
@pytest.mark.parametrize("form", [0, 1, 2])
def test_conv_halo_kernel_vs_torch_fp32(B, H, W, Cin, Cout, relu, with_res, form):
    """The halo-tiled 3x3 conv (mzba_conv_halo: config 3's 21x21 latent convs and 84x84 128 -> 256 conv; 256
    output pixels + W + 1 halo rows staged once per workgroup, every tap read from LDS, taps leaving the image
    redirected to a zero row) vs a torch fp32 conv of the same bf16 operands (+ bias, residual, ReLU), ragged
    pixel counts (the last tile partial), tiles crossing env boundaries; and close to conv_big_bf16_kernel.
    form (mzba_conv_halo_set_form): 0 the default (the 128-pixel two-workgroups-per-CU instance at W > 23, Cin =
    Cout = 256), 1 that instance wherever it fits, 2 the round-5 kernels; at W > 23 forms 0 / 1 equal form 2 bit for
    bit (the same two-block k order)."""
    from mzba import _lib as L
    from mzba.agent import pack_lat16
    assert L.lib().mzba_conv_halo_supported(H, W, Cin, Cout, 3)
    g = torch.Generator(device="cuda").manual_seed(B + Cin + W)
    dev = torch.device("cuda")
    x = torch.randn(B, H, W, Cin, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(Cout, 3, 3, Cin, generator=g, device=dev) / (Cin * 9) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, generator=g, device=dev)
    res = torch.randn(B, H, W, Cout, generator=g, device=dev).to(torch.bfloat16) if with_res else None
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=1)
    ref = ref.permute(0, 2, 3, 1) + (res.float() if with_res else 0)
    if relu:
        ref = torch.relu(ref)
    wh = torch.tensor(pack_lat16(w.float().cpu().numpy().reshape(Cout, -1), Cout, 3, Cin)).to(torch.bfloat16).cuda()
    out = torch.full((B, H, W, Cout), float("nan"), dtype=torch.bfloat16, device=dev)
    assert L.lib().mzba_conv_halo_set_form(form) == 0
    try:
        L.call("mzba_conv_halo", L.ptr(x), L.ptr(wh), L.ptr(b), L.ptr(res), L.ptr(out), B, H, W, Cin, Cout, relu,
               L.stream())
    finally:
        L.lib().mzba_conv_halo_set_form(0)
    big = torch.empty(B, H, W, Cout, dtype=torch.bfloat16, device=dev)
    L.call("mzba_conv2d", 1, L.ptr(x), H * W * Cin, None, 0, L.ptr(w), L.ptr(b), None, None, 0, L.ptr(res), L.ptr(big),
           B, H, W, Cin, Cout, 3, relu, L.stream())
    torch.cuda.synchronize()
    got = out.float()
    assert torch.isfinite(got).all()
    if W > 23 and Cin == Cout == 256 and form != 2:  # the 128-pixel form where the default takes it: round-5 bits
        o2 = torch.empty_like(out)
        assert L.lib().mzba_conv_halo_set_form(2) == 0
        try:
            L.call("mzba_conv_halo", L.ptr(x), L.ptr(wh), L.ptr(b), L.ptr(res), L.ptr(o2), B, H, W, Cin, Cout, relu,
                   L.stream())
        finally:
            L.lib().mzba_conv_halo_set_form(0)
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int16), o2.view(torch.int16))
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    print(f"conv_halo {B}x{H}x{W} {Cin}->{Cout}: max err {err / scale:.2e} of the magnitude, vs conv_big "
          f"{(got - big.float()).abs().max().item() / scale:.2e}")
    assert err <= 1e-2 * scale  # bf16 output rounding
    assert (got - big.float()).abs().max().item() <= 1e-2 * scale


@pytest.mark.parametrize("B,S,A", [(37, 5, 3), (150, 1, 3), (9, 50, 4)])
@pytest.mark.parametrize("form", [0, 1])
def test_conv_halo_gather_action_bias_vs_torch_fp32(B, S, A, form):
    """mzba_conv_halo_ex as config 3's dynamics first conv (networks.py:117-122, 160): every env's input
    gathered from its slot of a latent pool ((S + 1) latents per env), the action planes folded into a
    [HW][A][Cout] bias table (agent.py _conv act_w), ReLU — vs a torch fp32 conv of the gathered bf16 operands
    + the table row of the env's action + bias, and vs conv_igemm (mzba_conv2d) on the same arguments."""
    from mzba import _lib as L
    from mzba.agent import pack_lat16
    H = W = 21
    Cin = Cout = 256
    HW = H * W
    assert L.lib().mzba_conv_halo_ex_supported(H, W, Cin, Cout, 3, 1)
    g = torch.Generator(device="cuda").manual_seed(B + S)
    dev = torch.device("cuda")
    pool = torch.randn(B, S + 1, H, W, Cin, generator=g, device=dev).to(torch.bfloat16)
    slot = torch.randint(0, S + 1, (B,), generator=g, device=dev, dtype=torch.int32)
    act = torch.randint(0, A, (B,), generator=g, device=dev, dtype=torch.int32)
    w = (torch.randn(Cout, 3, 3, Cin, generator=g, device=dev) / (Cin * 9) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, generator=g, device=dev)
    tab = torch.randn(HW, A, Cout, generator=g, device=dev)
    x = pool[torch.arange(B, device=dev), slot.long()]
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=1)
    ref = ref.permute(0, 2, 3, 1) + tab[:, act.long()].permute(1, 0, 2).reshape(B, H, W, Cout)
    ref = torch.relu(ref)
    wh = torch.tensor(pack_lat16(w.float().cpu().numpy().reshape(Cout, -1), Cout, 3, Cin)).to(torch.bfloat16).cuda()
    out = torch.full((B, H, W, Cout), float("nan"), dtype=torch.bfloat16, device=dev)
    assert L.lib().mzba_conv_halo_set_form(form) == 0
    try:
        L.call("mzba_conv_halo_ex", L.ptr(pool), (S + 1) * HW * Cin, L.ptr(slot), HW * Cin, L.ptr(wh), L.ptr(b),
               L.ptr(tab), L.ptr(act), A, None, L.ptr(out), B, H, W, Cin, Cout, 1, L.stream())
    finally:
        L.lib().mzba_conv_halo_set_form(0)
    ig = torch.empty(B, H, W, Cout, dtype=torch.bfloat16, device=dev)
    L.call("mzba_conv2d", 1, L.ptr(pool), (S + 1) * HW * Cin, L.ptr(slot), HW * Cin, L.ptr(w), L.ptr(b), L.ptr(tab),
           L.ptr(act), A, None, L.ptr(ig), B, H, W, Cin, Cout, 3, 1, L.stream())
    torch.cuda.synchronize()
    got = out.float()
    assert torch.isfinite(got).all()
    scale = ref.abs().max().item()
    err = (got - ref).abs().max().item()
    print(f"conv_halo_ex B={B} S={S}: max err {err / scale:.2e} of the magnitude, vs conv_igemm "
          f"{(got - ig.float()).abs().max().item() / scale:.2e}")
    assert err <= 1e-2 * scale  # bf16 output rounding
    assert (got - ig.float()).abs().max().item() <= 1e-2 * scale
    # the contract's refusals: an action-bias table with a residual, an unsupported geometry
    assert L.lib().mzba_conv_halo_ex(L.ptr(pool), (S + 1) * HW * Cin, L.ptr(slot), HW * Cin, L.ptr(wh), L.ptr(b),
                                     L.ptr(tab), L.ptr(act), A, L.ptr(out), L.ptr(out), B, H, W, Cin, Cout, 1,
                                     L.stream()) == -1
    assert not L.lib().mzba_conv_halo_ex_supported(4, 5, Cin, Cout, 3, 1)


@pytest.mark.parametrize("B,H,W,Cin,Cout", [(150, 21, 21, 256, 256), (5, 84, 84, 256, 256), (37, 21, 21, 256, 128),
                                            (6, 84, 84, 128, 128)])
@pytest.mark.parametrize("form", [0, 1])
def test_conv_halo_in_place_residual(B, H, W, Cin, Cout, form):
    """The halo conv written in place over its residual (out aliases res, as a residual block may run it) equals the
    out-of-place result bit for bit: every lane reads its own (pixel, channel) residual elements before it writes
    them. The grid's partial last tile has waves wholly past the last pixel at B = 150 (their action-bias env index
    is clamped to the last env, conv_halo.hip halo_epilogue)."""
    from mzba import _lib as L
    from mzba.agent import pack_lat16
    g = torch.Generator(device="cuda").manual_seed(B + W + Cout)
    dev = torch.device("cuda")
    x = torch.randn(B, H, W, Cin, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(Cout, 3, 3, Cin, generator=g, device=dev) / (Cin * 9) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, generator=g, device=dev)
    res = torch.randn(B, H, W, Cout, generator=g, device=dev).to(torch.bfloat16)
    wh = torch.tensor(pack_lat16(w.float().cpu().numpy().reshape(Cout, -1), Cout, 3, Cin)).to(torch.bfloat16).cuda()
    out = torch.full((B, H, W, Cout), float("nan"), dtype=torch.bfloat16, device=dev)
    assert L.lib().mzba_conv_halo_set_form(form) == 0
    try:
        L.call("mzba_conv_halo", L.ptr(x), L.ptr(wh), L.ptr(b), L.ptr(res), L.ptr(out), B, H, W, Cin, Cout, 1,
               L.stream())
        inplace = res.clone()
        L.call("mzba_conv_halo", L.ptr(x), L.ptr(wh), L.ptr(b), L.ptr(inplace), L.ptr(inplace), B, H, W, Cin, Cout, 1,
               L.stream())
    finally:
        L.lib().mzba_conv_halo_set_form(0)
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all()
    assert torch.equal(out.view(torch.int16), inplace.view(torch.int16))


@pytest.mark.parametrize("B,ga", [(150, False), (37, True)])
def test_conv_halo_four_waves_equal_eight(B, ga):
    """mzba_conv_halo_set_waves(4) (one wave per SIMD, 128 pixels x 128 channels each: the round-5 A/B form of the
    Cin 256 one-block instances) gives the 8-wave outputs bit for bit, plain with a residual and gathered with an
    action-bias table (each accumulator takes its taps in the same order); other wave counts are refused."""
    from mzba import _lib as L
    from mzba.agent import pack_lat16
    H = W = 21
    C, A, S = 256, 3, 2
    HW = H * W
    g = torch.Generator(device="cuda").manual_seed(B + 7)
    dev = torch.device("cuda")
    pool = torch.randn(B, S + 1, H, W, C, generator=g, device=dev).to(torch.bfloat16)
    slot = torch.randint(0, S + 1, (B,), generator=g, device=dev, dtype=torch.int32)
    act = torch.randint(0, A, (B,), generator=g, device=dev, dtype=torch.int32)
    w = (torch.randn(C, 3, 3, C, generator=g, device=dev) / (C * 9) ** 0.5).to(torch.bfloat16)
    b = torch.randn(C, generator=g, device=dev)
    tab = torch.randn(HW, A, C, generator=g, device=dev)
    res = torch.randn(B, H, W, C, generator=g, device=dev).to(torch.bfloat16)
    wh = torch.tensor(pack_lat16(w.float().cpu().numpy().reshape(C, -1), C, 3, C)).to(torch.bfloat16).cuda()
    x = pool[:, 0].contiguous()
    outs = []
    try:
        for nw in (8, 4):
            assert L.lib().mzba_conv_halo_set_waves(nw) == 0
            o = torch.full((B, H, W, C), float("nan"), dtype=torch.bfloat16, device=dev)
            if ga:
                L.call("mzba_conv_halo_ex", L.ptr(pool), (S + 1) * HW * C, L.ptr(slot), HW * C, L.ptr(wh), L.ptr(b),
                       L.ptr(tab), L.ptr(act), A, None, L.ptr(o), B, H, W, C, C, 1, L.stream())
            else:
                L.call("mzba_conv_halo", L.ptr(x), L.ptr(wh), L.ptr(b), L.ptr(res), L.ptr(o), B, H, W, C, C, 1, L.stream())
            outs.append(o)
    finally:
        L.lib().mzba_conv_halo_set_waves(0)
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0].float()).all()
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
    assert L.lib().mzba_conv_halo_set_waves(6) == -1


@pytest.mark.parametrize("B,H,W,Cin,Cout,relu,with_res,same_order",
                         [(1000, 4, 5, 256, 256, 1, True, True), (37, 4, 5, 256, 256, 0, False, True),
                          (7, 16, 20, 128, 256, 1, True, True), (3, 21, 21, 256, 256, 1, True, True),
                          (512, 16, 20, 256, 256, 1, True, False), (512, 16, 20, 128, 128, 1, True, True)])
def test_conv_x6_is_as_close_to_exact_as_f32(B, H, W, Cin, Cout, relu, with_res, same_order):
    """mzba_conv_x6 (the f32 parity path's latent convs as six split-bf16 MFMA products each) against an f64
    conv of the same f32 operands: at least as close as the f32-input MFMA conv of the f32 path (mzba_conv2d
    dtype 0) — within 2x its error + 1e-7 of the magnitude — and within 2e-6 of the magnitude absolutely
    (ragged tiles, tiles crossing envs, every tap that leaves the image); the pre-split form (variant 1) and the
    per-read-split kernel bit-identical where both sum (tap, channel step) in order (same_order); round 5's 16x20
    instances: Cin 256 staged in two 128-channel blocks (160-pixel tiles; sums (block, tap, step): within 4e-6 of
    the per-read-split kernel), Cout 128 (the representation's 128-channel blocks; no per-read-split twin, the A/B
    variant 0 runs the same instance)."""
    from mzba import _lib as L
    from mzba.agent import split_pack_x6
    assert L.lib().mzba_conv_x6_supported(H, W, Cin, Cout, 3)
    g = torch.Generator(device="cuda").manual_seed(B + Cin + W)
    dev = torch.device("cuda")
    x = torch.rand(B, H, W, Cin, generator=g, device=dev)
    w = torch.randn(Cout, 3, 3, Cin, generator=g, device=dev) / (Cin * 9) ** 0.5
    b = torch.randn(Cout, generator=g, device=dev) * 0.1
    res = torch.rand(B, H, W, Cout, generator=g, device=dev) if with_res else None
    ref = torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), b.double(),
                                     padding=1).permute(0, 2, 3, 1)
    if with_res:
        ref = ref + res.double()
    if relu:
        ref = torch.relu(ref)
    wx = split_pack_x6(w.cpu().numpy().reshape(Cout, -1), Cout, 3, Cin).cuda()
    out = torch.full((B, H, W, Cout), float("nan"), device=dev)
    try:  # the pre-split form (variant 1; the default may pick the pixel-tiled form at 4x5, tested on its own below)
        assert L.lib().mzba_conv_x6_set_variant(1) == 0
        L.call("mzba_conv_x6", L.ptr(x), L.ptr(wx), L.ptr(b), L.ptr(res), L.ptr(out), B, H, W, Cin, Cout, relu,
               L.stream())
    finally:
        L.lib().mzba_conv_x6_set_variant(2)
    # the per-read-split kernel (the fallback where the pre-split form's rows do not fit): the same sums in the same order
    out2 = torch.full((B, H, W, Cout), float("nan"), device=dev)
    try:
        assert L.lib().mzba_conv_x6_set_variant(0) == 0
        L.call("mzba_conv_x6", L.ptr(x), L.ptr(wx), L.ptr(b), L.ptr(res), L.ptr(out2), B, H, W, Cin, Cout, relu, L.stream())
    finally:
        L.lib().mzba_conv_x6_set_variant(2)
    f32 = torch.empty(B, H, W, Cout, device=dev)
    wd = w.reshape(Cout, -1).contiguous()
    L.call("mzba_conv2d", 0, L.ptr(x), H * W * Cin, None, 0, L.ptr(wd), L.ptr(b), None, None, 0, L.ptr(res), L.ptr(f32),
           B, H, W, Cin, Cout, 3, relu, L.stream())
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    scale = ref.abs().max().item()
    if same_order:
        assert torch.equal(out, out2)
    else:
        assert (out - out2).abs().max().item() <= 4e-6 * scale
    e6, e32 = (out.double() - ref).abs().max().item(), (f32.double() - ref).abs().max().item()
    print(f"conv_x6 {B}x{H}x{W} {Cin}: max err vs f64 {e6 / scale:.2e} of the magnitude, f32 MFMA conv {e32 / scale:.2e}")
    assert e6 <= 2 * e32 + 1e-7 * scale and e6 <= 2e-6 * scale, (e6 / scale, e32 / scale)


@pytest.mark.parametrize("B,Cout,mode,ks", [(4100, 256, "res", 3), (37, 256, "plain", 3), (4096, 128, "plain", 3),
                                            (1000, 256, "gather", 3), (21, 128, "gather", 3), (4096, 256, "plain", 1),
                                            (45, 128, "plain", 1)])
def test_conv_x6_pixel_tiled_is_as_close_to_exact_as_f32(B, Cout, mode, ks):
    """The pixel-tiled x6 conv at the 4x5 latent (conv_x6t: 16 envs x 20 pixels per workgroup, the zero-padding
    taps not issued, the input staged in 32-channel blocks by LDS-DMA) against an f64 conv of the same f32
    operands: within 2x the f32-input MFMA conv's error + 1e-7 and within 2e-6 of the magnitude, and within 4e-6
    of the pre-split form (the same products summed in another order: the sum of two such errors). Ragged batches
    (B % 16 != 0), Cout 128 (the policy head's conv), the gathered form (each env's image read from a slot of a
    latent pool with the action planes' folded [HW][A][Cout] bias table, (acc + act_bias) + bias: the f32
    dynamics' first conv), and ks = 1 (the reward / value heads' 1x1 ConvBlocks: the centre tap only)."""
    from mzba import _lib as L
    from mzba.agent import split_pack_x6
    H, W, Cin, A, S = 4, 5, 256, 3, 6
    g = torch.Generator(device="cuda").manual_seed(B + Cout)
    dev = torch.device("cuda")
    w = torch.randn(Cout, ks, ks, Cin, generator=g, device=dev) / (Cin * ks * ks) ** 0.5
    b = torch.randn(Cout, generator=g, device=dev) * 0.1
    wx = split_pack_x6(w.cpu().numpy().reshape(Cout, -1), Cout, ks, Cin).cuda()
    relu = 1 if mode != "plain" else 0
    res = tab = act = slot = None
    if mode == "gather":
        pool = torch.rand(B, S + 1, H, W, Cin, generator=g, device=dev)
        slot = torch.randint(0, S + 1, (B,), generator=g, device=dev, dtype=torch.int32)
        act = torch.randint(0, A, (B,), generator=g, device=dev, dtype=torch.int32)
        tab = torch.randn(H * W, A, Cout, generator=g, device=dev) * 0.1
        x = pool[torch.arange(B, device=dev), slot.long()].contiguous()
        src, env_stride, slot_stride = pool, (S + 1) * H * W * Cin, H * W * Cin
    else:
        x = torch.rand(B, H, W, Cin, generator=g, device=dev)
        src, env_stride, slot_stride = x, H * W * Cin, 0
        if mode == "res":
            res = torch.rand(B, H, W, Cout, generator=g, device=dev)
    ref = torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), b.double(),
                                     padding=ks // 2).permute(0, 2, 3, 1)
    if res is not None:
        ref = ref + res.double()
    if tab is not None:
        ref = ref + tab.double()[:, act.long()].permute(1, 0, 2).reshape(B, H, W, Cout)
    if relu:
        ref = torch.relu(ref)
    assert L.lib().mzba_conv_x6_ex_supported(H, W, Cin, Cout, ks, int(mode == "gather"))
    out = torch.full((B, H, W, Cout), float("nan"), device=dev)
    try:
        assert L.lib().mzba_conv_x6_set_variant(3) == 0
        L.call("mzba_conv_x6_ex", L.ptr(src), env_stride, L.ptr(slot), slot_stride, L.ptr(wx), L.ptr(b), L.ptr(tab),
               L.ptr(act), A if tab is not None else 0, L.ptr(res), L.ptr(out), B, H, W, Cin, Cout, ks, relu, L.stream())
    finally:
        L.lib().mzba_conv_x6_set_variant(2)
    # the f32-input MFMA conv (conv_igemm, the f32 path's form before x6) on the same gathered operands
    f32 = torch.empty(B, H, W, Cout, device=dev)
    wd = w.reshape(Cout, -1).contiguous()
    L.call("mzba_conv2d", 0, L.ptr(src), env_stride, L.ptr(slot), slot_stride, L.ptr(wd), L.ptr(b), L.ptr(tab), L.ptr(act),
           A if tab is not None else 0, L.ptr(res), L.ptr(f32), B, H, W, Cin, Cout, ks, relu, L.stream())
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    scale = ref.abs().max().item()
    et, e32 = (out.double() - ref).abs().max().item(), (f32.double() - ref).abs().max().item()
    msg = f"conv_x6t B={B} Cout={Cout} {mode}: max err vs f64 {et / scale:.2e} of the magnitude, f32 MFMA conv {e32 / scale:.2e}"
    if mode != "gather" and Cout == 256 and ks == 3:  # the pre-split halo form on the same contiguous operands
        try:
            assert L.lib().mzba_conv_x6_set_variant(1) == 0
            outp = torch.full_like(out, float("nan"))
            L.call("mzba_conv_x6", L.ptr(x), L.ptr(wx), L.ptr(b), L.ptr(res), L.ptr(outp), B, H, W, Cin, Cout, relu,
                   L.stream())
        finally:
            L.lib().mzba_conv_x6_set_variant(2)
        torch.cuda.synchronize()
        ep = (out - outp).abs().max().item()
        msg += f", vs the pre-split form {ep / scale:.2e}"
        assert ep <= 4e-6 * scale, msg  # each within ~2e-6 of f64: apart by up to the sum
    print(msg)
    assert et <= 2 * e32 + 1e-7 * scale and et <= 2e-6 * scale, msg
    # the 4-wave (64-channel) and 8-wave (128-channel) workgroups: per 16-channel tile the same arithmetic, so the
    # same bits (the auto choice takes 4 waves where the 8-wave grid leaves CUs idle, e.g. config 2's 1 024 envs)
    outs = []
    try:
        for nw in (8, 4):
            assert L.lib().mzba_conv_x6_set_waves(nw) == 0 and L.lib().mzba_conv_x6_set_variant(3) == 0
            o = torch.full_like(out, float("nan"))
            L.call("mzba_conv_x6_ex", L.ptr(src), env_stride, L.ptr(slot), slot_stride, L.ptr(wx), L.ptr(b), L.ptr(tab),
                   L.ptr(act), A if tab is not None else 0, L.ptr(res), L.ptr(o), B, H, W, Cin, Cout, ks, relu, L.stream())
            outs.append(o)
    finally:
        L.lib().mzba_conv_x6_set_waves(0)
        L.lib().mzba_conv_x6_set_variant(2)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], out)
    assert L.lib().mzba_conv_x6_set_waves(6) == -1


@pytest.mark.parametrize("B,Cout,mode,ks,wspread", [(4100, 256, "res", 3, 0), (37, 256, "plain", 3, 0),
                                                    (4096, 128, "plain", 3, 0), (1000, 256, "gather", 3, 0),
                                                    (21, 128, "gather", 3, 0), (4096, 256, "plain", 1, 0),
                                                    (45, 128, "plain", 1, 0), (512, 256, "res", 3, 8),
                                                    (64, 128, "gather", 3, 8)])
def test_conv_x3_pixel_tiled_is_as_close_to_exact_as_f32(B, Cout, mode, ks, wspread):
    """Round 6: the split-fp16 x3 form of the pixel-tiled conv (mzba_conv_x3_ex: x = fp16 hi + fp16 lo, three fp16 MFMA
    products per f32 product, weights scaled by 2^k per output channel) against an f64 conv of the same f32 operands,
    on conv_x6t's cases (ragged batches, Cout 128, the gathered + action-biased form, 1x1): within 2x the f32-input MFMA
    conv's error + 2e-7 and within 3e-6 of the magnitude, and within 5e-6 of the x6 form. wspread: output channels
    whose weights differ in magnitude by up to 2^wspread (BN-folded weights of trained nets), each kept to 22 bits by
    its own 2^k. 8- and 4-wave workgroups bit-identical."""
    from mzba import _lib as L
    from mzba.agent import split_pack_x6, split_pack_x3
    H, W, Cin, A, S = 4, 5, 256, 3, 6
    g = torch.Generator(device="cuda").manual_seed(B + Cout + 7)
    dev = torch.device("cuda")
    w = torch.randn(Cout, ks, ks, Cin, generator=g, device=dev) / (Cin * ks * ks) ** 0.5
    if wspread:
        w = w * torch.exp2(torch.rand(Cout, 1, 1, 1, generator=g, device=dev) * wspread - wspread / 2)
    b = torch.randn(Cout, generator=g, device=dev) * 0.1
    wn = w.cpu().numpy().reshape(Cout, -1)
    wx = split_pack_x6(wn, Cout, ks, Cin).cuda()
    wx3, wsc = split_pack_x3(wn, Cout, ks, Cin)
    wx3, wsc = wx3.cuda(), wsc.cuda()
    relu = 1 if mode != "plain" else 0
    res = tab = act = slot = None
    if mode == "gather":
        pool = torch.rand(B, S + 1, H, W, Cin, generator=g, device=dev)
        slot = torch.randint(0, S + 1, (B,), generator=g, device=dev, dtype=torch.int32)
        act = torch.randint(0, A, (B,), generator=g, device=dev, dtype=torch.int32)
        tab = torch.randn(H * W, A, Cout, generator=g, device=dev) * 0.1
        x = pool[torch.arange(B, device=dev), slot.long()].contiguous()
        src, env_stride, slot_stride = pool, (S + 1) * H * W * Cin, H * W * Cin
    else:
        x = torch.rand(B, H, W, Cin, generator=g, device=dev)
        src, env_stride, slot_stride = x, H * W * Cin, 0
        if mode == "res":
            res = torch.rand(B, H, W, Cout, generator=g, device=dev)
    ref = torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), b.double(),
                                     padding=ks // 2).permute(0, 2, 3, 1)
    if res is not None:
        ref = ref + res.double()
    if tab is not None:
        ref = ref + tab.double()[:, act.long()].permute(1, 0, 2).reshape(B, H, W, Cout)
    if relu:
        ref = torch.relu(ref)
    assert L.lib().mzba_conv_x3_supported(H, W, Cin, Cout, ks, int(mode == "gather"))
    assert not L.lib().mzba_conv_x3_supported(H, W, Cin, Cout, 1, 1) and not L.lib().mzba_conv_x3_supported(8, 10, 128, 256, 3, 0)

    def run(fn, wts, extra=()):
        o = torch.full((B, H, W, Cout), float("nan"), device=dev)
        L.call(fn, L.ptr(src), env_stride, L.ptr(slot), slot_stride, L.ptr(wts), *extra, L.ptr(b), L.ptr(tab), L.ptr(act),
               A if tab is not None else 0, L.ptr(res), L.ptr(o), B, H, W, Cin, Cout, ks, relu, L.stream())
        return o
    out = run("mzba_conv_x3_ex", wx3, (L.ptr(wsc),))
    try:
        assert L.lib().mzba_conv_x6_set_variant(3) == 0
        out6 = run("mzba_conv_x6_ex", wx)
    finally:
        L.lib().mzba_conv_x6_set_variant(2)
    f32 = torch.empty(B, H, W, Cout, device=dev)
    wd = w.reshape(Cout, -1).contiguous()
    L.call("mzba_conv2d", 0, L.ptr(src), env_stride, L.ptr(slot), slot_stride, L.ptr(wd), L.ptr(b), L.ptr(tab), L.ptr(act),
           A if tab is not None else 0, L.ptr(res), L.ptr(f32), B, H, W, Cin, Cout, ks, relu, L.stream())
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    scale = ref.abs().max().item()
    e3, e6, e32 = [(o.double() - ref).abs().max().item() for o in (out, out6, f32)]
    d36 = (out - out6).abs().max().item()
    msg = (f"conv_x3t B={B} Cout={Cout} {mode} ks={ks} spread={wspread}: max err vs f64 {e3 / scale:.2e} of the "
           f"magnitude (x6 {e6 / scale:.2e}, f32 MFMA conv {e32 / scale:.2e}), vs x6 {d36 / scale:.2e}")
    print(msg)
    assert e3 <= 2 * e32 + 2e-7 * scale and e3 <= 3e-6 * scale, msg
    assert d36 <= 5e-6 * scale, msg
    outs = []
    try:  # 8 / 4 waves, and the pipelined split (default) against the split phase: the same sums, the same bits
        for nw, pipe in ((8, 1), (4, 1), (8, 0), (4, 0), (0, 2)):
            assert L.lib().mzba_conv_x6_set_waves(nw) == 0 and L.lib().mzba_conv_x3_set_pipe(pipe) == 0
            outs.append(run("mzba_conv_x3_ex", wx3, (L.ptr(wsc),)))
    finally:
        L.lib().mzba_conv_x6_set_waves(0)
        L.lib().mzba_conv_x3_set_pipe(1)
    torch.cuda.synchronize()
    assert all(torch.equal(o, out) for o in outs)
    assert L.lib().mzba_conv_x3_set_pipe(3) == -1


def test_f32_runner_defaults_to_x3_and_the_switch_reaches_new_runners():
    """The f32 agent's runners take the x3 convs by default (NetPack int use_x3 = 1) wherever a conv carries x3 weights
    — the latent towers, dyn0, the heads' convs and the representation's 3x3 convs — and NetPack.set_int('use_x3', 0)
    before a batch's first op gives that batch's runner the x6 convs."""
    from mzba.agent import MuZeroAgent, NetRunner
    cfg = default_config()
    ag = MuZeroAgent(cfg["model"], dtype="f32")
    ag.load_state_dict(init_state_dict(cfg["model"], 1))
    p = ag.packed
    assert all(c.get("wx3") is not None for blk in p.dyn + p.pred for c in blk)
    rep_3x3 = [c for kind, layer in p.rep if kind != "pool" for c in ([layer] if kind == "conv" else list(layer))
               if c["ks"] == 3 and c["cout"] % 128 == 0 and c["cin"] in (128, 256)]
    assert rep_3x3 and all(c.get("wx3") is not None for c in rep_3x3)
    assert NetRunner(p, 8, 16, 20).use_x3
    p.native.set_int("use_x3", 0)
    assert not NetRunner(p, 9, 16, 20).use_x3
    p.native.set_int("use_x3", 1)


def test_conv_x3_out_of_range_activation_is_loud():
    """The x3 form's one precondition: activations below 65 520 in magnitude (fp16's range). Past it the
    hi part is inf and the products turn non-finite (inf / NaN), so a violation shows as non-finite outputs at every
    position whose receptive field holds the value — never as a finite wrong number — while every other env is
    unaffected."""
    from mzba import _lib as L
    from mzba.agent import split_pack_x3
    B, H, W, C = 40, 4, 5, 256
    g = torch.Generator(device="cuda").manual_seed(5)
    dev = torch.device("cuda")
    x = torch.rand(B, H, W, C, generator=g, device=dev)
    x[3, 1, 2, 7] = 7.0e4
    w = torch.randn(C, 3, 3, C, generator=g, device=dev) / 48.0
    b = torch.zeros(C, device=dev)
    wx3, wsc = split_pack_x3(w.cpu().numpy().reshape(C, -1), C, 3, C)
    wx3, wsc = wx3.cuda(), wsc.cuda()
    out = torch.zeros(B, H, W, C, device=dev)
    L.call("mzba_conv_x3_ex", L.ptr(x), H * W * C, None, 0, L.ptr(wx3), L.ptr(wsc), L.ptr(b), None, None, 0, None,
           L.ptr(out), B, H, W, C, C, 3, 0, L.stream())
    torch.cuda.synchronize()
    assert not torch.isfinite(out[3, 0:3, 1:4]).any()  # the 3x3 neighbourhood of pixel (1, 2)
    mask = torch.ones(B, dtype=torch.bool, device=dev)
    mask[3] = False
    assert torch.isfinite(out[mask]).all()


@pytest.mark.parametrize("B,H,W,Cin,Cout,relu,with_res", [(7, 16, 20, 128, 256, 1, True), (512, 16, 20, 256, 256, 1, True),
                                                      (300, 16, 20, 128, 128, 1, False), (37, 8, 10, 256, 256, 0, False),
                                                      (1000, 8, 10, 256, 256, 1, True)])
def test_conv_x3_presplit_tiles_as_close_to_exact_as_f32(B, H, W, Cin, Cout, relu, with_res):
    """Round 6: the x3 form on the pre-split halo tiles (conv_x6p_kernel<.., NP = 2>, the f32 path's 16x20 and 8x10
    representation convs through mzba_conv_x3_ex) against an f64 conv of the same f32 operands: within 2x the
    f32-input MFMA conv's error + 2e-7 and within 3e-6 of the magnitude, within 5e-6 of the x6 form; ragged tiles,
    tiles crossing envs, every tap that leaves the image, weights differing by 2^6 between output channels."""
    from mzba import _lib as L
    from mzba.agent import split_pack_x6, split_pack_x3
    assert L.lib().mzba_conv_x3_supported(H, W, Cin, Cout, 3, 0) and not L.lib().mzba_conv_x3_supported(H, W, Cin, Cout, 3, 1)
    g = torch.Generator(device="cuda").manual_seed(B + Cin + W + 3)
    dev = torch.device("cuda")
    x = torch.rand(B, H, W, Cin, generator=g, device=dev)
    w = torch.randn(Cout, 3, 3, Cin, generator=g, device=dev) / (Cin * 9) ** 0.5
    w = w * torch.exp2(torch.rand(Cout, 1, 1, 1, generator=g, device=dev) * 6 - 3)
    b = torch.randn(Cout, generator=g, device=dev) * 0.1
    res = torch.rand(B, H, W, Cout, generator=g, device=dev) if with_res else None
    ref = torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(0, 3, 1, 2), b.double(),
                                     padding=1).permute(0, 2, 3, 1)
    if with_res:
        ref = ref + res.double()
    if relu:
        ref = torch.relu(ref)
    wn = w.cpu().numpy().reshape(Cout, -1)
    wx3, wsc = split_pack_x3(wn, Cout, 3, Cin)
    wx3, wsc = wx3.cuda(), wsc.cuda()
    wx = split_pack_x6(wn, Cout, 3, Cin).cuda()
    out = torch.full((B, H, W, Cout), float("nan"), device=dev)
    L.call("mzba_conv_x3_ex", L.ptr(x), H * W * Cin, None, 0, L.ptr(wx3), L.ptr(wsc), L.ptr(b), None, None, 0, L.ptr(res),
           L.ptr(out), B, H, W, Cin, Cout, 3, relu, L.stream())
    out6 = torch.full_like(out, float("nan"))
    L.call("mzba_conv_x6", L.ptr(x), L.ptr(wx), L.ptr(b), L.ptr(res), L.ptr(out6), B, H, W, Cin, Cout, relu, L.stream())
    f32 = torch.empty(B, H, W, Cout, device=dev)
    wd = w.reshape(Cout, -1).contiguous()
    L.call("mzba_conv2d", 0, L.ptr(x), H * W * Cin, None, 0, L.ptr(wd), L.ptr(b), None, None, 0, L.ptr(res), L.ptr(f32),
           B, H, W, Cin, Cout, 3, relu, L.stream())
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    scale = ref.abs().max().item()
    e3, e6, e32 = [(o.double() - ref).abs().max().item() for o in (out, out6, f32)]
    d36 = (out - out6).abs().max().item()
    msg = (f"conv_x3 pre-split {B}x{H}x{W} {Cin}->{Cout}: max err vs f64 {e3 / scale:.2e} of the magnitude (x6 "
           f"{e6 / scale:.2e}, f32 MFMA conv {e32 / scale:.2e}), vs x6 {d36 / scale:.2e}")
    print(msg)
    assert e3 <= 2 * e32 + 2e-7 * scale and e3 <= 3e-6 * scale, msg
    assert d36 <= 5e-6 * scale, msg


# ------------------------------------------------------------------------------ MCTS
@pytest.mark.parametrize("tag", ["b16_s50", "b4_s200"])
def test_mcts_replay_bit_exact(tag):
    from mzba.search import replay_search
    d = np.load(os.path.join(GOLDEN, f"mcts_{tag}.npz"))
    cfg = default_config()
    B, S = int(d["B"]), int(d["S"])
    values, counts, leaf = replay_search(B, S, cfg, d["v_root"], d["pi_root"], d["noise"], d["r"], d["v"], d["pi"],
                                         int(d["seed"]), int(d["search_id"]))
    np.testing.assert_array_equal(leaf, d["leaf_action"])
    np.testing.assert_array_equal(counts, d["counts"])
    np.testing.assert_array_equal(values.view(np.uint32), d["values"].view(np.uint32))


def test_dirichlet_noise_statistics():
    from mzba.search import TreeState
    from mzba import _lib as L
    B = 65536
    t = TreeState(B, 2, 1.25, 19652.0, "cuda")
    ta = t.args(0, 5, 1234)
    t.root(ta, torch.zeros(B, device="cuda"), torch.full((B, 3), 1 / 3, device="cuda"), None, 0.825, 0.175, 0.25)
    n = t.noise.cpu().numpy().astype(np.float64)
    assert np.all(n >= 0) and np.allclose(n.sum(1), 1, atol=1e-5)
    # Dirichlet(0.25,0.25,0.25): mean 1/3, var = (1/3)(2/3)/(0.75+1) = 0.12698
    assert abs(n.mean() - 1 / 3) < 5e-3
    assert abs(n[:, 0].var() - (2 / 9) / 1.75) < 5e-3
    # determinism: same (seed, search id) -> same noise
    n2 = t.noise.clone()
    t.root(ta, torch.zeros(B, device="cuda"), torch.full((B, 3), 1 / 3, device="cuda"), None, 0.825, 0.175, 0.25)
    assert torch.equal(n2, t.noise)
    del L


def _sample_dev(counts, T, step, seed, inv_t_dev=None, n_total=None, off=0, vb=32, threads=1):
    from mzba import _lib as L
    B = counts.shape[0]
    a = torch.empty(B, dtype=torch.int64, device="cuda")
    p = torch.empty(B, 3, dtype=torch.float32, device="cuda")
    cd = dev(counts)
    L.call("mzba_sample_actions", L.ptr(cd), L.ptr(a), L.ptr(p), B, 1.0 / T, L.ptr(inv_t_dev),
           off + B if n_total is None else n_total, vb, threads, off, step, seed, None, L.stream())
    torch.cuda.synchronize()
    return a.cpu().numpy(), p.cpu().numpy()


def test_sample_kernel_matches_reference_fixture():
    """Temperature sampling bit-exact against the reference's own `visit_counts ** (1/T)` / sum
    (train_torch.py:192-193, torch CPU, tests/golden/sampling.npz): probabilities (uint32 view) and
    the inverse-CDF action, for 18 temperatures (the reference's decay schedule incl. the 0.1 floor,
    and the special exponents 2 and 4) and every lane class of torch's CPU pow (B = 4096, 1029, 12, 2)."""
    d = np.load(os.path.join(GOLDEN, "sampling.npz"))
    seed, vb = int(d["seed"]), int(d["vec_block"])
    for name in ("b4096", "b1029", "b12", "b2"):
        counts = d[f"{name}/counts"]
        for i, T in enumerate(d["temps"]):
            act, probs = _sample_dev(counts, float(T), i, seed, vb=vb)
            np.testing.assert_array_equal(probs.view(np.uint32), d[f"{name}/t{i}/probs"].view(np.uint32),
                                          err_msg=f"{name} T={T}")
            np.testing.assert_array_equal(act, d[f"{name}/t{i}/action"], err_msg=f"{name} T={T}")


def test_sample_kernel_device_temperature_and_shards():
    """1/T read from the device buffer (graph-replayable) == the launch argument; a shard
    (env_offset, global n_envs_total) takes the lanes of its global positions: the two halves of
    the B = 1029 fixture batch equal the whole."""
    d = np.load(os.path.join(GOLDEN, "sampling.npz"))
    seed = int(d["seed"])
    counts = d["b1029/counts"]
    i = 9
    T = float(d["temps"][i])
    ref_a, ref_p = d[f"b1029/t{i}/action"], d[f"b1029/t{i}/probs"]
    inv = torch.tensor([1.0 / T], dtype=torch.float64, device="cuda")
    a, p = _sample_dev(counts, 1.0, i, seed, inv_t_dev=inv)
    np.testing.assert_array_equal(p.view(np.uint32), ref_p.view(np.uint32))
    np.testing.assert_array_equal(a, ref_a)
    for off, n in ((0, 515), (515, 514)):
        a, p = _sample_dev(counts[off:off + n], T, i, seed, n_total=1029, off=off)
        np.testing.assert_array_equal(p.view(np.uint32), ref_p[off:off + n].view(np.uint32))
        np.testing.assert_array_equal(a, ref_a[off:off + n])


def test_torch_pow_device_exhaustive():
    """The device pow (csrc/torch_pow.h) against torch's CPU results over counts 0..1023 at every
    exponent of the reference's temperature schedule, SLEEF vector lanes and scalar (double pow)
    lanes (fixture checksums) and element for element against the oracle's C restatement."""
    from mzba import _lib as L
    from oracle.torch_pow import pow_counts
    d = np.load(os.path.join(GOLDEN, "sampling.npz"))
    base = np.arange(1024, dtype=np.int64)
    bd = dev(base)
    out = torch.empty(1024, dtype=torch.float32, device="cuda")
    for j, T in enumerate(d["sched_temps"]):
        for n_total, key in ((4096, "sched_pow_vec_u32sum"), (1024 + 3, "sched_pow_scalar_u32sum")):
            # rows at positions [0, 1024) of a 4096-element tensor: all vector lanes; at positions
            # [0, 1024) of a 1027-element tensor with vb = 2048: all scalar lanes
            vb = 32 if n_total == 4096 else 2048
            L.call("mzba_torch_pow", L.ptr(bd), L.ptr(out), 1024, 1.0 / T, 0, n_total, vb, 1, L.stream())
            got = out.cpu().numpy()
            assert got.view(np.uint32).astype(np.uint64).sum() == d[key][j], (T, key)
            ref = pow_counts(base[:, None], 1.0 / T, vb, 0, n_total // 3 if n_total == 4096 else 1)[:, 0]
            np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32), err_msg=f"T={T} {key}")


def test_sample_kernel_threaded_pow_chunks():
    """From 32768 elements on torch's CPU pow runs in per-thread chunks, each with its own scalar tail
    (TensorIterator::for_each -> at::parallel_for), so the lane of an element depends on the reference
    process's thread count: 12000 envs (36000 elements; a 2-thread chunk of 18000 is not a multiple of
    32) at 1 / 2 / 3 / 8 threads — the device pow equals torch's own `counts ** (1/T)` computed here with
    that many threads, and the sampled probabilities / actions equal the oracle's, shards included."""
    from mzba import _lib as L
    from oracle.acting import sample_actions, sample_probs
    from oracle import rng as R
    n_env, T, seed, step = 12000, 0.996 ** 37, 3, 5
    counts = np.random.default_rng(1).integers(0, 51, (n_env, 3))
    cd = dev(counts)
    out = torch.empty(3 * n_env, dtype=torch.float32, device="cuda")
    nthreads = torch.get_num_threads()
    try:
        for thr in (1, 2, 3, 8):
            torch.set_num_threads(thr)
            ref = (torch.from_numpy(counts) ** (1.0 / T)).numpy().reshape(-1)
            L.call("mzba_torch_pow", L.ptr(cd), L.ptr(out), 3 * n_env, 1.0 / T, 0, 3 * n_env, 32, thr, L.stream())
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32), err_msg=f"{thr} threads")
            a, p = _sample_dev(counts, T, step, seed, threads=thr)
            u = R.uniform(np.arange(n_env), R.STREAM_SAMPLE, step, 0, seed)
            np.testing.assert_array_equal(p.view(np.uint32), sample_probs(counts, T, threads=thr).view(np.uint32))
            np.testing.assert_array_equal(a, sample_actions(counts, T, u, threads=thr))
            for off, n in ((0, 7001), (7001, 4999)):  # shards take the lanes of their global positions
                a2, p2 = _sample_dev(counts[off:off + n], T, step, seed, n_total=n_env, off=off, threads=thr)
                np.testing.assert_array_equal(p2.view(np.uint32), p[off:off + n].view(np.uint32))
    finally:
        torch.set_num_threads(nthreads)


def _replay_reference_episode(name, graph):
    """A reference `_run_episode` fixture through ActingLoop (small f32 nets, the fixture's own
    Dirichlet noise injected, keyed reset / tie-break / sampling streams)."""
    from mzba.agent import MuZeroAgent
    from mzba.acting import ActingLoop
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    cfg = _small_cfg(50)
    mcfg = cfg["model"]
    seed, B = int(d["seed"]), int(d["B"])
    T = float(d["temperature"]) if "temperature" in d.files else 1.0
    sd = init_state_dict(mcfg, seed)
    ag = MuZeroAgent(mcfg, dtype="f32")
    ag.load_state_dict(sd)
    loop = ActingLoop(cfg, ag, B, seed=seed, temperature=T)
    loop.inject_noise = lambda sid, n: d["noise"][sid]
    trajs = loop.run_episode(0)
    return d, trajs, mcfg["state_history_length"]


@pytest.mark.parametrize("name", ["acting_small_b4", "acting_small_b12_t150"])
def test_acting_loop_replays_reference_episode(name):
    """SURVEY §8(a) rows 1-18 end to end against the reference's own `_run_episode` (tests/golden,
    generated by importing /root/reference): actions, visit counts, rewards and grayscale frames
    bit-exact, values within the f32 net tolerance. b12_t150 runs at the decayed temperature
    0.996**150 (torch's SLEEF lanes and scalar lanes both in play)."""
    d, trajs, L_ = _replay_reference_episode(name, graph=False)
    for b, t in enumerate(trajs):
        n = int(d["lengths"][b])
        assert t.length == n, (b, t.length, n)
        np.testing.assert_array_equal(np.array(t.actions[L_:]), d["actions"][b, :n])
        np.testing.assert_array_equal(np.stack([c.numpy() for c in t.visit_counts[L_:]]), d["counts"][b, :n])
        np.testing.assert_array_equal(np.array(t.rewards[L_:], np.float32), d["rewards"][b, :n])
        np.testing.assert_array_equal(np.stack([s.numpy() for s in t.states[L_ - 1:]]).reshape(n, 16, 20),
                                      d["frames"][b, :n])
        np.testing.assert_allclose(np.array(t.values[L_:], np.float32), d["values"][b, :n], rtol=1e-4, atol=1e-5)


def test_dropin_classes_replay_reference_episode():
    """The drop-in classes driven exactly like the reference's `_run_episode` (train_torch.py:171-233:
    environment.parallel_breakout.BreakoutEnvironment.step, MuZeroAgent.create_hidden_state_root,
    MCTSSearchVec.search, the reference's CPU sampling and recording) reproduce its fixture."""
    from environment.parallel_breakout import BreakoutEnvironment
    from src.networks import MuZeroAgent
    from src.mcts import MCTSSearchVec
    d = np.load(os.path.join(GOLDEN, "acting_small_b12_t150.npz"))
    cfg = _small_cfg(50)
    mcfg = cfg["model"]
    seed, B, T = int(d["seed"]), int(d["B"]), float(d["temperature"])
    L_ = mcfg["state_history_length"]
    env = BreakoutEnvironment({**cfg["environment"], "n_parallel": B}, seed=seed)
    ag = MuZeroAgent(mcfg, dtype="f32")
    ag.load_state_dict(init_state_dict(mcfg, seed))
    ag.eval_mode()
    search = MCTSSearchVec(cfg, ag, None, seed=seed)
    state, _ = env.reset()
    gray = convert_to_grayscale(state.cpu().numpy())
    trajs = [Trajectory(L_, gray[b]) for b in range(B)]
    done = torch.zeros(B, dtype=torch.bool)
    prev_done = done
    warp = gray
    t = 0
    while not bool(done.all()) and t <= 260:
        x = np.stack([prepare_mcts_input(warp[b], trajs[b], L_) for b in range(B)])
        h = ag.create_hidden_state_root(dev(x))
        values, counts = search.search(h, torch.ones(B, 3), 0, noise=d["noise"][t])
        u = R.uniform(np.arange(B), R.STREAM_SAMPLE, t, 0, seed)
        action = sample_actions(counts.numpy(), T, u)
        state, reward, done, valid = env.step(state, torch.from_numpy(action), done)
        warp = convert_to_grayscale(state.cpu().numpy())
        for b in range(B):
            if not bool(prev_done[b]):
                trajs[b].add_observation(action[b], warp[b], float(reward[b]), counts.numpy()[b], float(values[b]))
        prev_done = done.clone()
        t += 1
    for b, tr in enumerate(trajs):
        n = int(d["lengths"][b])
        assert tr.length == n
        np.testing.assert_array_equal(np.array(tr.actions[L_:]), d["actions"][b, :n])
        np.testing.assert_array_equal(np.stack(tr.visit_counts[L_:]), d["counts"][b, :n])
        np.testing.assert_array_equal(np.array(tr.rewards[L_:], np.float32), d["rewards"][b, :n])
        np.testing.assert_array_equal(np.stack(tr.states[L_ - 1:]).reshape(n, 16, 20), d["frames"][b, :n])


def test_run_test_simulation_matches_reference():
    """mzba.acting.run_test_simulation against the reference's own
    RLSystem.run_test_simulation(batch=2) (tests/golden/test_sim_b2.npz: learner net for the root,
    target net in the search, T = 0.1, padding action 1, env 0's action recorded for every env)."""
    from mzba.agent import MuZeroAgent
    from mzba.acting import run_test_simulation
    d = np.load(os.path.join(GOLDEN, "test_sim_b2.npz"))
    cfg = _small_cfg(50)
    mcfg = cfg["model"]
    B, seed = int(d["B"]), int(d["seed"])
    tgt, lrn = MuZeroAgent(mcfg, dtype="f32"), MuZeroAgent(mcfg, dtype="f32")
    tgt.load_state_dict(init_state_dict(mcfg, int(d["target_seed"])))
    lrn.load_state_dict(init_state_dict(mcfg, int(d["learner_seed"])))
    import mzba.acting as A
    orig = A.ActingLoop.__init__

    def init(self, *a, **k):
        orig(self, *a, **k)
        self.inject_noise = lambda sid, n: d["noise"][sid]
    A.ActingLoop.__init__ = init
    try:
        trajs, frames, _ = run_test_simulation(cfg, tgt, batch=B, seed=seed, rep_agent=lrn)
    finally:
        A.ActingLoop.__init__ = orig
    L_ = mcfg["state_history_length"]
    n = int(d["n_steps"])
    for b, t in enumerate(trajs):
        assert t.length == n
        np.testing.assert_array_equal(np.array(t.actions), d["actions"][b])
        np.testing.assert_array_equal(np.stack([c.numpy() for c in t.visit_counts[L_:]]), d["counts"][b])
        np.testing.assert_array_equal(np.array(t.rewards[L_:], np.float32), d["rewards"][b])
        np.testing.assert_array_equal(np.stack([s.numpy() for s in t.states[L_ - 1:]]).reshape(n, 16, 20),
                                      d["states"][b])
        np.testing.assert_allclose(np.array(t.values[L_:], np.float32), d["values"][b], rtol=1e-4, atol=1e-5)
    np.testing.assert_array_equal(np.stack([f.numpy() for f in frames[0]]).reshape(-1, 16, 20), d["env0_frames"])


def _small_cfg(S):
    cfg = default_config()
    cfg["model"] = small_model_cfg(cfg)
    cfg["num_simulations"] = S
    return cfg


def test_search_f32_matches_oracle():
    """Full 50-sim searches on the f32 path (nets on the GPU) vs the numpy oracle's nets + dict trees,
    same keyed noise and tie-breaks. The tree arithmetic is bit-exact (replay tests); the nets agree to
    1e-5, which can flip a PUCT decision that is tied to that precision. Stated bound: at most 1 of
    the 16 envs may end with different visit counts, and where counts agree the root values agree to
    rtol 1e-4 / atol 1e-5."""
    from mzba.agent import MuZeroAgent
    from mzba.search import MCTSSearchVec
    cfg = _small_cfg(50)
    mcfg = cfg["model"]
    sd = init_state_dict(mcfg, 7)
    ag = MuZeroAgent(mcfg, dtype="f32")
    ag.load_state_dict(sd)
    B = 16
    x = np.random.default_rng(3).random((B, 8, 16, 20)).astype(np.float32)
    h = N.create_hidden_state_root(x, sd, mcfg)
    s = MCTSSearchVec(cfg, ag, None, seed=42)
    s.search_id = 3
    values, counts = s.search(dev(h), torch.ones(B, 3), 0)
    noise = s._ws[list(s._ws)[0]].tree.noise.cpu().numpy()
    o = MCTSOracle(cfg, NetModel(sd, mcfg), 42)
    ov, oc = o.search(h, noise, 3)
    match = (counts.numpy() == oc).all(1).mean()
    assert match >= 15 / 16, (match, counts.numpy(), oc)
    np.testing.assert_allclose(values.numpy()[(counts.numpy() == oc).all(1)], ov[(counts.numpy() == oc).all(1)],
                               rtol=1e-4, atol=1e-5)


def test_acting_loop_f32_matches_oracle_episode():
    from mzba.agent import MuZeroAgent
    from mzba.acting import ActingLoop
    cfg = _small_cfg(20)
    mcfg = cfg["model"]
    sd = init_state_dict(mcfg, 5)
    ag = MuZeroAgent(mcfg, dtype="f32")
    ag.load_state_dict(sd)
    B, seed = 8, 2024
    loop = ActingLoop(cfg, ag, B, seed=seed, max_steps=30)
    loop.noise_log = []
    trajs = loop.run_episode(0)
    noises = [n.cpu().numpy() for n in loop.noise_log]
    otrajs, _ = run_episode(cfg, sd, seed, 0, lambda sid, n: noises[sid], B, max_steps=30)
    L_ = mcfg["state_history_length"]
    for b in range(B):
        assert trajs[b].length == otrajs[b].length
        np.testing.assert_array_equal(trajs[b].actions, otrajs[b].actions)
        np.testing.assert_array_equal(np.stack([c.numpy() for c in trajs[b].visit_counts[L_:]]),
                                      np.stack(otrajs[b].visit_counts[L_:]) if otrajs[b].length else np.zeros((0, 3)))
        np.testing.assert_array_equal(np.array(trajs[b].rewards[L_:], np.float32), np.array(otrajs[b].rewards[L_:], np.float32))
        np.testing.assert_array_equal(np.stack([s.numpy() for s in trajs[b].states]), np.stack(otrajs[b].states))
        np.testing.assert_allclose(trajs[b].values[L_:], np.array(otrajs[b].values[L_:], np.float32), rtol=1e-4, atol=1e-5)


def test_full_size_bf16_acting_step_vs_f32_path():
    """BASELINE config 2's workload end to end under -m gpu: one acting step of 1024 envs x 50 sims with
    the full-width bf16 nets (the benchmarked path: fused towers, tree update in the prediction launch)
    against the same step on the f32 parity path (same state, same keyed noise and tie-breaks).
    Stated bound: bf16 rounding in the 2 x 14-block towers moves close PUCT decisions, so at least
    85 % of envs must have identical visit counts (measured: 0.92 on 64 envs against the f32 CPU port,
    bench visit_count_match); every count row sums to S; where counts agree, the root values agree
    within 0.05 absolute (bf16 value logits)."""
    from mzba.agent import MuZeroAgent
    from mzba.acting import ActingLoop
    cfg = default_config()
    cfg["num_simulations"] = 50
    sd = init_state_dict(cfg["model"], 0)
    out = {}
    for dt in ("bf16", "f32"):
        ag = MuZeroAgent(cfg["model"], dtype=dt)
        ag.load_state_dict(sd)
        loop = ActingLoop(cfg, ag, 1024, seed=5)
        loop.reset(0)
        loop.act(eager=True)
        torch.cuda.synchronize()
        out[dt] = {k: v[0].cpu().numpy() for k, v in loop.rec.items() if v is not None}
        del loop, ag
        torch.cuda.empty_cache()
    c16, c32 = out["bf16"]["counts"], out["f32"]["counts"]
    assert (c16.sum(1) == 50).all() and (c32.sum(1) == 50).all()
    same = (c16 == c32).all(1)
    print("bf16 vs f32 visit-count agreement at 1024 x 50:", same.mean())
    assert same.mean() >= 0.85, same.mean()
    assert np.abs(out["bf16"]["values"][same] - out["f32"]["values"][same]).max() <= 0.05


def test_acting_loop_84x84_config3_geometry_matches_oracle():
    """BASELINE config 3's geometry as a parity case: 84x84 frames (parallel_breakout.py reads
    self.height / self.width everywhere), 4-frame stack (8 input planes), latent 21x21 after the
    two avg-pools, reduced-width f32 nets; trajectories, visit counts, rewards and frames equal
    the oracle's run_episode at the same size (injected noise)."""
    from mzba.agent import MuZeroAgent
    from mzba.acting import ActingLoop
    cfg = _small_cfg(8)
    mcfg = cfg["model"]
    mcfg["latent_resolution"] = [21, 21]
    sd = init_state_dict(mcfg, 11)
    ag = MuZeroAgent(mcfg, dtype="f32")
    ag.load_state_dict(sd)
    B, seed, T = 3, 77, 5
    loop = ActingLoop(cfg, ag, B, seed=seed, max_steps=T, height=84, width=84)
    loop.noise_log = []
    trajs = loop.run_episode(0)
    noises = [n.cpu().numpy() for n in loop.noise_log]
    otrajs, _ = run_episode(cfg, sd, seed, 0, lambda sid, n: noises[sid], B, max_steps=T, height=84, width=84)
    L_ = mcfg["state_history_length"]
    for b in range(B):
        assert trajs[b].length == otrajs[b].length
        np.testing.assert_array_equal(trajs[b].actions, otrajs[b].actions)
        np.testing.assert_array_equal(np.stack([c.numpy() for c in trajs[b].visit_counts[L_:]]),
                                      np.stack(otrajs[b].visit_counts[L_:]) if otrajs[b].length else np.zeros((0, 3)))
        np.testing.assert_array_equal(np.array(trajs[b].rewards[L_:], np.float32), np.array(otrajs[b].rewards[L_:], np.float32))
        np.testing.assert_array_equal(np.stack([s.numpy() for s in trajs[b].states]), np.stack(otrajs[b].states))
        np.testing.assert_allclose(trajs[b].values[L_:], np.array(otrajs[b].values[L_:], np.float32), rtol=1e-4, atol=1e-5)


def _pack_wf(wp, cout):
    K = wp.shape[1]
    wf = wp.reshape(cout // 32, 32, K // 16, 2, 8).transpose(0, 2, 3, 1, 4).reshape(-1)
    return np.concatenate([wf, np.zeros(8 * 64 * 8, wf.dtype)])


@pytest.mark.parametrize("B,H,W,Cin,Cout,ks", [(7, 4, 5, 256, 256, 3), (1024, 4, 5, 256, 256, 3), (9, 4, 5, 256, 128, 3),
                                                (512, 4, 5, 256, 256, 3), (511, 4, 5, 128, 256, 1),
                                                (13, 4, 5, 256, 256, 1), (5, 8, 10, 256, 256, 3), (3, 4, 5, 64, 64, 3),
                                                (17, 4, 5, 64, 32, 1), (4, 8, 10, 128, 128, 3)])
def test_conv_lat_vs_torch(B, H, W, Cin, Cout, ks):
    """conv_lat (LDS-resident activations, fragment-major weights) vs torch fp32 conv, with
    the slot gather, the per-(pixel, action) bias and the residual all exercised."""
    from mzba import _lib as L
    g = torch.Generator().manual_seed(B * 7 + Cout)
    S1 = 3
    pool = torch.randn(B, S1, H, W, Cin, generator=g).to(torch.bfloat16)
    slot = torch.randint(0, S1, (B,), generator=g, dtype=torch.int32)
    w = torch.randn(Cout, Cin, ks, ks, generator=g) / (Cin * ks * ks) ** 0.5
    b = torch.randn(Cout, generator=g)
    A = 3
    act = torch.randint(0, A, (B,), generator=g, dtype=torch.int32)
    ab = torch.randn(H * W, A, Cout, generator=g)
    res = torch.randn(B, H, W, Cout, generator=g).to(torch.bfloat16)
    x = pool[torch.arange(B), slot.long()].float()  # (B,H,W,Cin)
    wq = w.to(torch.bfloat16).float()
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), wq, b, padding=ks // 2).permute(0, 2, 3, 1)
    ref = torch.relu(ref + ab.view(H, W, A, Cout)[:, :, act.long()].permute(2, 0, 1, 3) + res.float())
    wp = w.permute(0, 2, 3, 1).reshape(Cout, -1).numpy()
    from mzba.agent import pack_lat
    wf = torch.from_numpy(pack_lat(wp, Cout, ks, Cin)).to(torch.bfloat16).cuda()
    out = torch.empty(B, H, W, Cout, dtype=torch.bfloat16, device="cuda")
    assert L.lib().mzba_conv_lat_supported(H, W, Cin, Cout, ks) == 1
    d = {k: v.cuda() for k, v in dict(pool=pool, slot=slot, b=b, ab=ab, act=act, res=res).items()}  # keep alive
    L.call("mzba_conv_lat", L.ptr(d["pool"]), S1 * H * W * Cin, L.ptr(d["slot"]), H * W * Cin, L.ptr(wf),
           L.ptr(d["b"]), L.ptr(d["ab"]), L.ptr(d["act"]), A, L.ptr(d["res"]), L.ptr(out), B, H, W, Cin,
           Cout, ks, 1, L.stream())
    err = (out.float().cpu() - ref).abs().max().item() / max(1.0, ref.abs().max().item())
    assert err < 1e-2, err
    # 3-row-tile workgroups (chosen where the 5-tile grid leaves CUs idle) vs 5-tile ones: the
    # per-element arithmetic is the same, so the outputs are bit-identical
    out5 = torch.empty_like(out)
    L.call("mzba_conv_lat_set_variant", 2)
    try:
        L.call("mzba_conv_lat", L.ptr(d["pool"]), S1 * H * W * Cin, L.ptr(d["slot"]), H * W * Cin, L.ptr(wf),
               L.ptr(d["b"]), L.ptr(d["ab"]), L.ptr(d["act"]), A, L.ptr(d["res"]), L.ptr(out5), B, H, W, Cin,
               Cout, ks, 1, L.stream())
    finally:
        L.call("mzba_conv_lat_set_variant", 0)
    assert torch.equal(out, out5)


def test_acting_graph_replay_matches_eager():
    """One captured HIP graph per acting step, replayed: identical records to eager launches."""
    from mzba.agent import MuZeroAgent
    from mzba.acting import ActingLoop
    cfg = _small_cfg(8)
    mcfg = cfg["model"]
    sd = init_state_dict(mcfg, 9)
    ag = MuZeroAgent(mcfg, dtype="bf16")
    ag.load_state_dict(sd)
    out = []
    for graph in (False, True):
        loop = ActingLoop(cfg, ag, 64, seed=77, max_steps=12)
        loop.reset(0)
        loop.act(eager=True)
        if graph:
            loop.capture()
        for _ in range(11):
            loop.act()
        torch.cuda.synchronize()
        out.append({k: v.cpu().numpy() for k, v in loop.rec.items() if v is not None})
    for k in out[0]:
        np.testing.assert_array_equal(out[0][k], out[1][k], err_msg=k)


def test_acting_graph_replays_across_the_schedule():
    """The step graph captured at T = 1, noise weight 0.175 keeps replaying correctly after the train
    loop's schedule moves (train_torch.py:129-135: T *= 0.996, noise_weight = 0.1): 1/T and the
    root mixing weights are device values, so replayed steps equal eager steps at the new settings."""
    from mzba.agent import MuZeroAgent
    from mzba.acting import ActingLoop
    cfg = _small_cfg(8)
    sd = init_state_dict(cfg["model"], 9)
    ag = MuZeroAgent(cfg["model"], dtype="bf16")
    ag.load_state_dict(sd)
    out = []
    for graph in (False, True):
        loop = ActingLoop(cfg, ag, 64, seed=78, max_steps=12)
        loop.reset(0)
        loop.act(eager=True)
        if graph:
            loop.capture()
        for i in range(11):
            if i == 3:
                loop.temperature = 0.996 ** 40
                loop.search.noise_weight = 0.1
            loop.act()
        torch.cuda.synchronize()
        out.append({k: v.cpu().numpy() for k, v in loop.rec.items() if v is not None})
    for k in out[0]:
        np.testing.assert_array_equal(out[0][k], out[1][k], err_msg=k)


def test_sharded_loops_equal_global_loop():
    """Two shards (env_offset 0 and 8) reproduce the 16-env loop env for env: the RNG is keyed
    on the global env id, so results do not depend on the world size."""
    from mzba.agent import MuZeroAgent
    from mzba.acting import ActingLoop
    cfg = _small_cfg(6)
    sd = init_state_dict(cfg["model"], 3)
    ag = MuZeroAgent(cfg["model"], dtype="f32")
    ag.load_state_dict(sd)

    def run(B, off):  # T < 1: the shard's sampling takes the torch pow lanes of its global positions
        loop = ActingLoop(cfg, ag, B, seed=13, env_offset=off, max_steps=10, n_envs_total=16, temperature=0.8)
        loop.reset(0)
        for _ in range(10):
            loop.act(eager=True)
        torch.cuda.synchronize()
        return {k: v.cpu().numpy() for k, v in loop.rec.items() if v is not None}

    full = run(16, 0)
    parts = [run(8, 0), run(8, 8)]
    for k in full:
        np.testing.assert_array_equal(np.concatenate([parts[0][k], parts[1][k]], axis=1), full[k], err_msg=k)


def test_scalar_transforms_decode_kernel():
    from mzba.scalar import ScalarTransforms
    st = ScalarTransforms(default_config()["model"])
    x = torch.randn(37, 11)
    np.testing.assert_allclose(st.inverted_softmax_expectation(x).numpy(),
                               N.inverted_softmax_expectation(x.numpy()), rtol=1e-5, atol=1e-6)


def test_dropin_modules_resolve_via_get_class():
    """The reference's plugin boundary (utils.py:84-96, train_torch.py:86-94) loads this build."""
    from utils import get_class
    cfg = default_config()
    Env = get_class(cfg["environment"]["environment_path"], cfg["environment"]["environment_name"])
    Search = get_class("src.mcts", cfg["search"]["mcts_name"])
    Agent = get_class("src.networks", cfg["model"]["agent_name"])
    from mzba.env import BreakoutEnvironment
    from mzba.search import MCTSSearchVec
    from mzba.agent import MuZeroAgent
    assert Env is BreakoutEnvironment and Search is MCTSSearchVec and Agent is MuZeroAgent
    e = Env({**cfg["environment"], "n_parallel": 4})
    s, _ = e.reset()
    assert tuple(s.shape) == e.state_shape


@pytest.mark.parametrize("variant", [1, 2, 3, 4])
@pytest.mark.parametrize("B,nblocks,gather", [(4, 1, False), (13, 3, True), (1024, 2, False)])
def test_tower_matches_conv_chain(B, nblocks, gather, variant):
    """Fused tower (activations LDS-resident across blocks) vs torch fp32 residual blocks with
    bf16-rounded weights and bf16 intermediates."""
    from mzba import _lib as L
    from mzba.agent import pack_tower_conv
    g = torch.Generator().manual_seed(B + nblocks)
    C, H, W = 256, 4, 5
    S1 = 3 if gather else 1
    pool = torch.rand(B, S1, H, W, C, generator=g).to(torch.bfloat16)
    slot = torch.randint(0, S1, (B,), generator=g, dtype=torch.int32)
    ws = [torch.randn(C, C, 3, 3, generator=g) / (C * 9) ** 0.5 for _ in range(2 * nblocks)]
    bs = [torch.randn(C, generator=g) * 0.1 for _ in range(2 * nblocks)]
    x = pool[torch.arange(B), slot.long()].float().permute(0, 3, 1, 2)
    bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    for k in range(nblocks):
        t1 = bf(torch.relu(torch.nn.functional.conv2d(x, bf(ws[2 * k]), bs[2 * k], padding=1)))
        x = bf(torch.relu(torch.nn.functional.conv2d(t1, bf(ws[2 * k + 1]), bs[2 * k + 1], padding=1) + x))
    ref = x.permute(0, 2, 3, 1)
    L.call("mzba_tower_set_variant", variant)
    plan = L.lib().mzba_tower_plan(B)
    nb = L.lib().mzba_tower_ws_bytes(B)
    L.call("mzba_tower_set_variant", 0)
    assert plan == variant and nb == 0
    wsb = torch.zeros(max(nb, 16), dtype=torch.uint8, device="cuda")
    wf = np.concatenate([pack_tower_conv(w.numpy()) for w in ws]
                        + [np.zeros(8 * 64 * 8, np.float32)])
    d = dict(pool=pool.cuda(), slot=slot.cuda(), wf=torch.from_numpy(wf).to(torch.bfloat16).cuda(),
             b=torch.cat(bs).cuda())
    out = torch.empty(B, H, W, C, dtype=torch.bfloat16, device="cuda")
    L.call("mzba_tower_set_variant", variant)
    try:
        L.call("mzba_tower", L.ptr(d["pool"]), S1 * H * W * C, L.ptr(d["slot"]) if gather else None, H * W * C,
               L.ptr(out), L.ptr(d["wf"]), L.ptr(d["b"]), nblocks, B, L.ptr(wsb), nb, L.stream())
        torch.cuda.synchronize()
    finally:
        L.call("mzba_tower_set_variant", 0)
    err = (out.float().cpu() - ref).abs().max().item() / max(1.0, ref.abs().max().item())
    assert err < 3e-2, err


# ------------------------------------------------------------------------------ replay ingest
def _replay_oracle_from(trajs, cfg, max_length, nsum):
    from oracle.replay import ReplayOracle
    K, h = cfg["num_unroll_steps"], cfg["model"]["state_history_length"]
    o = ReplayOracle(h, K, max_length, cfg["discount_factor"], nsum)
    for t in trajs:
        if t.length > K + 1:  # train_torch.py:224
            o.save([int(a) for a in t.actions[h:]], np.stack([np.asarray(s).reshape(16, 20) for s in t.states[h - 1:]]),
                   np.asarray(t.states[0]).reshape(16, 20), np.array([float(r) for r in t.rewards[h:]], np.float32),
                   np.stack([np.asarray(c) for c in t.visit_counts[h:]]), np.array(t.values[h:], np.float32))
    return o


def _check_replay(buf, o):
    idx = torch.arange(len(o))
    assert len(buf) == len(o)
    np.testing.assert_array_equal(buf.get_batched_past_actions(idx).cpu().numpy(), o.batched("past_actions", idx))
    np.testing.assert_array_equal(buf.get_batched_future_actions(idx).cpu().numpy(), o.batched("future_actions", idx))
    np.testing.assert_array_equal(buf.get_batched_states(idx).cpu().numpy()[:, :, 0], o.batched("states", idx))
    np.testing.assert_array_equal(buf.get_batched_rewards(idx).cpu().numpy(), o.batched("rewards", idx))
    np.testing.assert_array_equal(buf.get_batched_visit_counts(idx).cpu().numpy(), o.batched("visit_counts", idx))
    np.testing.assert_array_equal(buf.get_values(idx).cpu().numpy(), o.batched("values", idx))
    np.testing.assert_array_equal(buf.get_batched_values(idx).cpu().numpy(), o.batched("targets", idx))
    np.testing.assert_array_equal(np.array(buf.get_reward_sums(), np.float32), o.reward_sums())


def test_replay_buffer_matches_reference_fixture():
    """Drop-in ReplayBuffer (device windows + n-step targets) vs the reference run on the same
    trajectories (tests/golden/replay.npz), including FIFO eviction: bit-exact."""
    from replay_buffer import ReplayBuffer, ObservationTrajectory
    d = np.load(os.path.join(GOLDEN, "replay.npz"))
    h, K = int(d["hist"]), int(d["K"])
    buf = ReplayBuffer(h, K, int(d["max_length"]), float(d["discount"]), int(d["num_rewards_to_sum"]))
    for i, L in enumerate(d["lengths"]):
        f0 = torch.from_numpy(d["frame0"][i].reshape(1, 16, 20))
        t = ObservationTrajectory([0] * h, [f0] * (h - 1), [0] * h, [torch.zeros(3)] * h, [0.0] * h, 0, 0)
        for s in range(L):
            t.add_observation(int(d["actions"][i, s]), torch.from_numpy(d["frames"][i, s].reshape(1, 16, 20)),
                              float(d["rewards"][i, s]), torch.from_numpy(d["counts"][i, s]), float(d["values"][i, s]))
        buf.save_observation_trajectory(t)
    idx = torch.arange(int(d["n"]))
    assert len(buf) == int(d["n"])
    np.testing.assert_array_equal(buf.get_batched_past_actions(idx).cpu().numpy(), d["past_actions"])
    np.testing.assert_array_equal(buf.get_batched_future_actions(idx).cpu().numpy(), d["future_actions"])
    np.testing.assert_array_equal(buf.get_batched_states(idx).cpu().numpy(), d["states"])
    np.testing.assert_array_equal(buf.get_batched_rewards(idx).cpu().numpy(), d["b_rewards"])
    np.testing.assert_array_equal(buf.get_batched_visit_counts(idx).cpu().numpy(), d["b_counts"])
    np.testing.assert_array_equal(buf.get_batched_values(idx).cpu().numpy(), d["targets"])
    np.testing.assert_array_equal(np.array(buf.get_reward_sums(), np.float32), d["reward_sums"])


@pytest.mark.parametrize("max_length", [100000, 97])
def test_replay_ingest_from_acting_records(max_length):
    """Device ingest straight from the acting loop's sink (no host trajectories) vs the oracle
    ReplayBuffer fed the same episode's ObservationTrajectory lists; small ring = eviction."""
    from mzba.agent import MuZeroAgent
    from mzba.acting import ActingLoop
    from mzba.replay import DeviceReplayBuffer
    cfg = _small_cfg(8)
    mcfg = cfg["model"]
    ag = MuZeroAgent(mcfg, dtype="bf16")
    ag.load_state_dict(init_state_dict(mcfg, 31))
    B = 48
    loop = ActingLoop(cfg, ag, B, seed=99, max_steps=40)
    trajs = loop.run_episode(0)
    K, h = cfg["num_unroll_steps"], mcfg["state_history_length"]
    buf = DeviceReplayBuffer(h, K, max_length, cfg["discount_factor"], 64)
    buf.ingest_records(loop.rec, loop.frame0.view(B, -1), loop.t)
    buf.ingest_records(loop.rec, loop.frame0.view(B, -1), loop.t)  # a second episode batch: FIFO order
    o = _replay_oracle_from(list(trajs) + list(trajs), cfg, max_length, 64)
    assert len(o) > 0
    _check_replay(buf, o)


def test_checkpoint_reference_format_roundtrip(tmp_path):
    """save_checkpoint writes RLSystem._save_weights' dict (train_torch.py:612-637); load_checkpoint
    (weights_only) restores the agent and the device replay buffer exactly."""
    from mzba.agent import MuZeroAgent
    from mzba.checkpoint import save_checkpoint, load_checkpoint, REPLAY_KEYS
    from replay_buffer import ReplayBuffer, ObservationTrajectory
    cfg = _small_cfg(8)
    mcfg = cfg["model"]
    ag = MuZeroAgent(mcfg, dtype="f32")
    ag.load_state_dict(init_state_dict(mcfg, 3))
    d = np.load(os.path.join(GOLDEN, "replay.npz"))
    h, K = int(d["hist"]), int(d["K"])
    buf = ReplayBuffer(h, K, int(d["max_length"]), float(d["discount"]), int(d["num_rewards_to_sum"]))
    for i, L in enumerate(d["lengths"]):
        f0 = torch.from_numpy(d["frame0"][i].reshape(1, 16, 20))
        t = ObservationTrajectory([0] * h, [f0] * (h - 1), [0] * h, [torch.zeros(3)] * h, [0.0] * h, 0, 0)
        for s in range(L):
            t.add_observation(int(d["actions"][i, s]), torch.from_numpy(d["frames"][i, s].reshape(1, 16, 20)),
                              float(d["rewards"][i, s]), torch.from_numpy(d["counts"][i, s]), float(d["values"][i, s]))
        buf.save_observation_trajectory(t)
    p = str(tmp_path / "checkpt.pth")
    save_checkpoint(p, ag, buf, training_iteration=7, acting_step=3, iteration=11)
    raw = torch.load(p, weights_only=True)
    assert set(raw) == {"model_state_dict", "optimizer_state_dict", "training_iteration", "acting_step", "iteration",
                        "replay_buffer"}
    assert set(raw["replay_buffer"]) == set(REPLAY_KEYS)
    # the reference's _load_weights does optimizer.load_state_dict(...) on Adam(mu_zero.parameters()):
    # the default-saved optimizer state must load into an Adam over parameters of those shapes
    from mzba.weights import state_dict_spec
    params = [torch.nn.Parameter(torch.zeros(s)) for k, s in state_dict_spec(mcfg)
              if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))]
    torch.optim.Adam(params, lr=mcfg["learning_rate"], weight_decay=1e-4).load_state_dict(raw["optimizer_state_dict"])
    np.testing.assert_array_equal(torch.stack(raw["replay_buffer"]["state_buffer"]).numpy(), d["states"])
    np.testing.assert_array_equal(torch.stack(raw["replay_buffer"]["bootstrapped_values"]).numpy(), d["targets"])
    ag2 = MuZeroAgent(mcfg, dtype="f32")
    buf2 = ReplayBuffer(h, K, int(d["max_length"]), float(d["discount"]), int(d["num_rewards_to_sum"]))
    ck = load_checkpoint(p, ag2, buf2)
    assert ck["training_iteration"] == 7 and ck["iteration"] == 11
    for k, v in ag.state_dict().items():
        np.testing.assert_array_equal(ag2.state_dict()[k], v)
    idx = torch.arange(len(buf))
    for get in ("get_batched_past_actions", "get_batched_future_actions", "get_batched_states", "get_batched_rewards",
                "get_batched_visit_counts", "get_batched_values"):
        assert torch.equal(getattr(buf, get)(idx), getattr(buf2, get)(idx)), get
    assert buf.get_reward_sums() == buf2.get_reward_sums()


@pytest.mark.parametrize("variant,S", [(1, 12), (2, 12), (3, 12), (2, 200), (3, 200), (4, 12), (4, 200)])
def test_tree_step_fused_into_prediction_is_identical(variant, S):
    """backup(sim) + select(sim + 1) inside the fused prediction launch == the separate tree
    kernels: same visit counts, values and tie-break draws, bit for bit (bf16 nets), at 12 and at
    config 5's 200 simulations (201-node trees)."""
    from mzba import _lib as L
    from mzba.agent import MuZeroAgent
    from mzba.search import MCTSSearchVec
    cfg = default_config()
    cfg["num_simulations"] = S
    mcfg = cfg["model"]
    ag = MuZeroAgent(mcfg, dtype="bf16")
    ag.load_state_dict(init_state_dict(mcfg, 4))
    B = 13
    g = torch.Generator().manual_seed(5)
    h = torch.rand(B, 256, 4, 5, generator=g).cuda()
    out = []
    L.call("mzba_tower_set_variant", variant)
    try:
        for fuse in (False, True):
            ag._runners = {}
            s = MCTSSearchVec(cfg, ag, None, seed=17)
            ws = s.workspace(B)
            ws.use_tree_fusion = fuse
            assert ws.runner.fused_ok() and ws.runner.tower_plan == variant
            v, c = s.search(h)
            out.append((v.numpy(), c.numpy()))
    finally:
        L.call("mzba_tower_set_variant", 0)
    np.testing.assert_array_equal(out[0][1], out[1][1])
    np.testing.assert_array_equal(out[0][0], out[1][0])


def test_test_simulation_matches_oracle():
    """run_test_simulation (train_torch.py:530-610) on the device vs the oracle restatement: padding
    action 1, T = 0.1 sampling, action[0] recorded for every env, frames while live (f32 nets)."""
    from mzba.agent import MuZeroAgent
    from mzba.acting import run_test_simulation
    from oracle.acting import run_test_simulation as oracle_test
    cfg = _small_cfg(12)
    mcfg = cfg["model"]
    sd = init_state_dict(mcfg, 8)
    ag = MuZeroAgent(mcfg, dtype="f32")
    ag.load_state_dict(sd)
    trajs, frames, loop = run_test_simulation(cfg, ag, batch=2, seed=55, max_steps_test=40, log_noise=True)
    noises = [n.cpu().numpy() for n in loop.noise_log]
    otrajs, oframes = oracle_test(cfg, sd, 55, 0, lambda sid, n: noises[sid], batch=2, max_steps_test=40)
    L_ = mcfg["state_history_length"]
    for b in range(2):
        assert trajs[b].length == otrajs[b].length
        np.testing.assert_array_equal(trajs[b].actions, otrajs[b].actions)
        np.testing.assert_array_equal(np.stack([s.numpy() for s in trajs[b].states]), np.stack(otrajs[b].states))
        np.testing.assert_array_equal(np.array(trajs[b].rewards[L_:], np.float32),
                                      np.array(otrajs[b].rewards[L_:], np.float32))
        np.testing.assert_array_equal(np.stack([c.numpy() for c in trajs[b].visit_counts[L_:]]),
                                      np.stack(otrajs[b].visit_counts[L_:]))
        assert len(frames[b]) == len(oframes[b])
        if frames[b]:
            np.testing.assert_array_equal(np.stack([f.numpy() for f in frames[b]]), np.stack(oframes[b]))


@pytest.mark.parametrize("B,variant", [(64, 1), (64, 3), (2048, 0), (4096, 4)])
def test_fp16_dynamics_step(B, variant):
    """BASELINE config 5's fp16 dynamics net: the fused dynamics step with fp16 LDS images / weights
    / MFMA (latents in and out bf16) against the f32 path of the same weights; its error must not
    exceed the all-bf16 step's (fp16 keeps 3 more mantissa bits)."""
    from mzba import _lib as L
    from mzba.agent import MuZeroAgent
    mcfg = default_config()["model"]
    sd = init_state_dict(mcfg, 9)
    S1, n = 3, 20 * 256
    g = torch.Generator().manual_seed(B + 1)
    pool0 = torch.rand(B, S1 + 1, n, generator=g).to(torch.bfloat16).cuda()
    slot = torch.randint(0, S1, (B,), generator=g, dtype=torch.int32).cuda()
    act = torch.randint(0, 3, (B,), generator=g, dtype=torch.int32).cuda()
    res = {}
    for tag, dt, dyn in (("f32", "f32", None), ("bf16", "bf16", None), ("fp16", "bf16", "fp16")):
        ag = MuZeroAgent(mcfg, dtype=dt, dyn_dtype=dyn)
        ag.load_state_dict(sd)
        L.call("mzba_tower_set_variant", variant)
        try:
            rn = ag.runner(B, 16, 20)
        finally:
            L.call("mzba_tower_set_variant", 0)
        tdt = torch.float32 if dt == "f32" else torch.bfloat16
        pool = pool0.to(tdt)
        out = torch.empty(B, n, dtype=tdt, device="cuda")
        r, rl = torch.full((B,), float("nan"), device="cuda"), torch.full((B, 11), float("nan"), device="cuda")
        if dyn:
            assert rn.fused_ok() and rn.tower_plan == (variant or 2)
        rn.dynamics(pool, act, out, r, rl, slot=slot, env_stride=(S1 + 1) * n, slot_stride=n, pool=pool,
                    pool_env_stride=(S1 + 1) * n, pool_slot=S1)
        torch.cuda.synchronize()
        res[tag] = [t.float().cpu() for t in (out, rl)]
    for i, nm in enumerate(("latent", "reward_logits")):
        e16 = (res["fp16"][i] - res["f32"][i]).abs().max().item()
        eb = (res["bf16"][i] - res["f32"][i]).abs().max().item()
        assert torch.isfinite(res["fp16"][i]).all() and e16 <= max(eb, 1e-2), (nm, e16, eb)


def test_f32_heads_bit_identical_to_their_sum_order():
    """mzba_heads (f32 parity path: the Linear heads + softmax / support decode, networks.py:138-149, 200-223,
    utils.py:74-81). The FMA form (variant 0) with several envs per workgroup (round 5: the weights read once per 8
    envs, not per env) keeps each env's f32 sum order: thread t accumulates k = t, t + 256, ... in sequence, the
    wave's xor-shuffle tree, then ((w0 + w1) + (w2 + w3)) + bias — the logits equal a numpy f32 emulation of exactly
    that order bit for bit (ragged B), two heads per launch (value: support decode; policy: softmax). The f32-MFMA
    form (default since round 5: 16 envs per workgroup, f32 products accumulated in f32 in 32 partial sums per
    output) is within 5e-7 of the magnitude of an f64 evaluation (an f32 sum of 2560-5120 products; the FMA form's
    tree lands ~1.2e-7 away)."""
    from mzba import _lib as L
    g = np.random.default_rng(5)
    B = 37
    heads = [(5120, 11, 1), (2560, 3, 0)]
    xs = [g.standard_normal((B, K)).astype(np.float32) for K, _, _ in heads]
    ws = [(g.standard_normal((O, K)) * 0.02).astype(np.float32) for K, O, _ in heads]
    bs = [g.standard_normal(O).astype(np.float32) * 0.1 for _, O, _ in heads]

    def emulate(x, w, b):
        O, K = w.shape
        out = np.zeros((x.shape[0], O), np.float32)
        for e in range(x.shape[0]):
            for o in range(O):
                part = np.zeros(256, np.float32)
                for k0 in range(0, K, 256):
                    part = (part + (x[e, k0:k0 + 256] * w[o, k0:k0 + 256]).astype(np.float32)).astype(np.float32)
                waves = []
                for wv in range(4):
                    v = part[64 * wv:64 * (wv + 1)].copy()
                    for s in (32, 16, 8, 4, 2, 1):
                        v = (v + v[np.arange(64) ^ s]).astype(np.float32)
                    waves.append(v[0])
                r = np.float32(np.float32(waves[0] + waves[1]) + np.float32(waves[2] + waves[3]))
                out[e, o] = np.float32(r + b[o])
        return out

    dx = [torch.as_tensor(x, device="cuda") for x in xs]
    dw = [torch.as_tensor(w, device="cuda") for w in ws]
    db = [torch.as_tensor(b, device="cuda") for b in bs]
    lg = [torch.empty(B, O, device="cuda") for _, O, _ in heads]
    dec = [torch.empty(B, device="cuda"), torch.empty(B, 3, device="cuda")]
    def run():
        L.call("mzba_heads", 0, 2, L.ptr(dx[0]), L.ptr(dw[0]), L.ptr(db[0]), 5120, 11, 1, L.ptr(lg[0]), L.ptr(dec[0]),
               L.ptr(dx[1]), L.ptr(dw[1]), L.ptr(db[1]), 2560, 3, 0, L.ptr(lg[1]), L.ptr(dec[1]), -5.0, 5.0, B,
               L.stream())
        torch.cuda.synchronize()
        return [t.clone() for t in lg], [t.clone() for t in dec]

    try:
        assert L.lib().mzba_heads_set_variant(0) == 0
        lg_fma, dec_fma = run()
    finally:
        L.lib().mzba_heads_set_variant(1)
    lg_mfma, dec_mfma = run()
    for i in range(2):
        want = emulate(xs[i], ws[i], bs[i])
        np.testing.assert_array_equal(lg_fma[i].cpu().numpy().view(np.uint32), want.view(np.uint32))
        exact = xs[i].astype(np.float64) @ ws[i].astype(np.float64).T + bs[i]
        scale = np.abs(exact).max()
        e_fma = np.abs(want - exact).max()
        e_mfma = np.abs(lg_mfma[i].cpu().numpy() - exact).max()
        assert e_mfma <= 5e-7 * scale, (i, e_mfma / scale, e_fma / scale)  # f32 sums of 2560-5120 products
    for dd, ll in ((dec_fma, lg_fma), (dec_mfma, lg_mfma)):
        torch.testing.assert_close(dd[1], torch.softmax(ll[1], 1), rtol=1e-6, atol=1e-7)
