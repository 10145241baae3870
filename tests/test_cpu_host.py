"""CPU-only checks of the host side: C-ABI library loads and exports every symbol
declared in include/mzba.h (no compute without a GPU), weight packing/spec logic."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from mzba.config import default_config, small_model_cfg
from mzba.weights import init_state_dict, state_dict_spec


def _declared():
    h = open(os.path.join(ROOT, "include", "mzba.h")).read()
    return sorted(set(re.findall(r"\b(mzba_[a-z0-9_]+)\s*\(", h)))


def test_library_exports_every_declared_symbol():
    from mzba import _lib
    L = _lib.lib()
    decl = _declared()
    assert decl, "no declarations parsed"
    for name in decl:
        assert hasattr(L, name), name
    assert sorted(_lib.exported_symbols()) == decl


def test_node_layout_is_one_line():
    from mzba import _lib
    assert _lib.lib().mzba_mcts_node_bytes() == 64


def test_bad_arguments_rejected_without_gpu():
    from mzba import _lib
    import ctypes
    rc = _lib.lib().mzba_conv2d(1, None, 0, None, 0, None, None, None, None, 0, None, None, 0, 4, 5, 256, 256, 3,
                                1, None)
    assert rc < 0
    rc = _lib.lib().mzba_conv2d(1, None, 0, None, 0, None, None, None, None, 0, None, None, 2, 4, 5, 100, 256, 3,
                                1, None)
    assert rc == -2
    del ctypes


def test_product_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from mzba.agent import MuZeroAgent
    with pytest.raises(RuntimeError):
        MuZeroAgent(default_config()["model"])


@pytest.mark.parametrize("small", [False, True])
def test_state_dict_spec_matches_reference_layout(small):
    cfg = default_config()
    m = small_model_cfg(cfg) if small else cfg["model"]
    spec = dict(state_dict_spec(m))
    c1 = m["latent_channels"][1]
    assert spec["dyn_net.conv_block.conv.weight"] == (c1, c1 + 3, 3, 3)
    assert spec["pred_net.value_head.2.weight"] == (11, c1 // 2 * 20)
    sd = init_state_dict(m, 0)
    assert len(sd) == len(spec)
    w = sd["rep_net.blocks.0.weight"]
    assert np.abs(w).max() <= 1 / np.sqrt(np.prod(w.shape[1:]))
    if not small:
        n = sum(int(np.prod(s)) for k, s in spec.items() if not k.endswith("num_batches_tracked"))
        assert n > 40_000_000  # rep 8.05M + dyn 17.26M + pred 16.90M


def test_ucb_tables_double_precision():
    import math
    import torch
    from mzba.search import ucb_tables
    sq, ct = ucb_tables(50, 1.25, 19652.0, "cpu")
    for n in (0, 1, 7, 50):
        assert sq[n].item() == float(np.float32(math.sqrt(n)))
        assert ct[n].item() == float(np.float32(1.25 + math.log((n + 19652.0 + 1) / 19652.0)))
    del torch


def test_torch_custom_ops_registered():
    """libmzba_torch.so registers TORCH_LIBRARY(mz) with the drop-in surface of SURVEY §8(b);
    env_step declares the reference's done_mask aliasing (Tensor(a!) done -> Tensor(a!))."""
    from mzba import _lib
    ops = _lib.ops()
    for name in _lib.TORCH_OPS:
        assert hasattr(ops, name), name
    sch = str(ops.env_step.default._schema)
    assert "Tensor(a!) done" in sch and "Tensor(a!) done_out" in sch, sch
    assert "Tensor(h!) values" in str(ops.mcts_results_.default._schema)


def test_net_ops_schemas_declare_their_writes():
    """The nets as custom ops (csrc/net_ops.cpp): the reference surface takes the weight pack
    (mz.NetPack) and returns new tensors; the NHWC acting forms and the fused prediction + tree step
    declare every buffer they write as Tensor(x!) — the tree buffers of prediction_tree_ included —
    and nothing they only read."""
    import torch
    from mzba import _lib
    ops = _lib.ops()
    assert "__torch__.torch.classes.mz.NetPack nets" in str(ops.representation.default._schema)
    for name, writes, reads in (
            ("dynamics_", ["out", "r_dec", "r_logits", "pool"], ["src", "act", "slot"]),
            ("prediction_", ["pi", "v", "p_logits", "v_logits"], ["h"]),
            ("prediction_tree_", ["pi", "v", "nodes", "root_sum", "calls", "leaf_parent", "leaf_action", "depth",
                                  "path"], ["h", "sqrt_tab", "c_tab", "r", "ctx"]),
            ("representation_", ["out", "pool"], ["x"])):
        args = {a.name: a for a in getattr(ops, name).default._schema.arguments}
        for w in writes:
            assert args[w].alias_info is not None and args[w].alias_info.is_write, (name, w)
        for r in reads:
            assert args[r].alias_info is None, (name, r)
    p = torch.classes.mz.NetPack()
    p.set_int("k", 7)
    assert p.get_int("k") == 7 and not p.fused_ok()


def test_default_checkpoint_optimizer_state_loads_into_reference_adam():
    """Without a learner, save_checkpoint writes a fresh Adam state that the reference's
    `optimizer.load_state_dict` (train_torch.py:646) accepts: one group, every parameter."""
    import torch
    from mzba.checkpoint import fresh_optimizer_state
    from mzba.config import default_config
    from mzba.weights import state_dict_spec
    mcfg = default_config()["model"]
    params = [torch.nn.Parameter(torch.zeros(1)) for k, _ in state_dict_spec(mcfg)
              if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))]
    opt = torch.optim.Adam(params, lr=mcfg["learning_rate"], weight_decay=1e-4)
    opt.load_state_dict(fresh_optimizer_state(mcfg))
    assert opt.param_groups[0]["weight_decay"] == 1e-4 and len(opt.param_groups[0]["params"]) == len(params)


def test_scale_division_by_double_reciprocal_is_ieee():
    """towerp.hip's _scale_state divides (h - min) by den = (max - min) + 1e-8 as
    f32((double)(h - min) * f64(1 / den)); that must be the IEEE f32 quotient bit for bit (the
    product is within 2^-52 of the exact quotient, a quotient of two f32 at least 2^-49 from a
    rounding midpoint). Checked on 4M random pairs over the ranges the scale sees plus edge pairs."""
    rng = np.random.default_rng(3)
    a = np.concatenate([rng.random(2_000_000, dtype=np.float32) * np.float32(37.0),
                        rng.random(2_000_000, dtype=np.float32) * np.float32(1e-3),
                        np.array([0.0, 1.0, 3.0, 1e-8, 65504.0], np.float32)])
    d = np.concatenate([rng.random(2_000_000, dtype=np.float32) * np.float32(37.0) + np.float32(1e-8),
                        rng.random(2_000_000, dtype=np.float32) * np.float32(1e-3) + np.float32(1e-8),
                        np.array([1e-8, 3.0, 3.0, 7.0, 3.0], np.float32)]).astype(np.float32)
    q_ieee = a / d
    q_dbl = (a.astype(np.float64) * (1.0 / d.astype(np.float64))).astype(np.float32)
    np.testing.assert_array_equal(q_ieee.view(np.uint32), q_dbl.view(np.uint32))


def test_rep_trunk_rejects_bad_arguments_without_gpu():
    """mzba_rep_trunk checks its arguments before any HIP call: null buffers or pointer tables, negative
    block counts, more convs than its kernel-argument tables hold (2 n0 + 2 + 2 n1 <= 56), in == out."""
    import ctypes
    from mzba import _lib
    L = _lib.lib()
    nc = 2 * 2 + 2 + 2 * 3
    w = (ctypes.c_void_p * nc)(*([1] * nc))
    b = (ctypes.c_void_p * nc)(*([1] * nc))
    x, y = ctypes.c_void_p(16), ctypes.c_void_p(32)
    assert L.mzba_rep_trunk(None, y, w, b, 2, 3, 4, None) == -1
    assert L.mzba_rep_trunk(x, y, None, b, 2, 3, 4, None) == -1
    assert L.mzba_rep_trunk(x, y, w, b, -1, 3, 4, None) == -1
    assert L.mzba_rep_trunk(x, y, w, b, 2, 3, 0, None) == -1
    assert L.mzba_rep_trunk(x, x, w, b, 2, 3, 4, None) == -1
    assert L.mzba_rep_trunk(x, y, w, b, 20, 8, 4, None) == -1  # 58 convs
    wn = (ctypes.c_void_p * nc)(*([1] * (nc - 1) + [0]))
    assert L.mzba_rep_trunk(x, y, wn, b, 2, 3, 4, None) == -1


@pytest.mark.parametrize("tag", ["small", "full"])
def test_agent_random_init_equals_reference_construction(tag):
    """MuZeroAgent(cfg)'s starting weights (networks.py:245-266) are the reference agent's bit for
    bit under the same torch seed: tests/golden/agent_init.npz holds per-tensor checksums of the
    reference's own `MuZeroAgent(cfg)` built twice in a row (RLSystem's learner and target agents,
    train_torch.py:86-88) after torch.manual_seed(42) (train_torch.py set_seed) and (7)."""
    import torch
    from conftest import GOLDEN
    from mzba.weights import torch_init_state_dict
    d = np.load(os.path.join(GOLDEN, "agent_init.npz"))
    mcfg = small_model_cfg() if tag == "small" else default_config()["model"]
    for seed in (42, 7):
        torch.manual_seed(seed)
        for ai in range(2):
            sd = torch_init_state_dict(mcfg)
            assert list(sd) == [k for k, _ in state_dict_spec(mcfg)]
            for k, v in sd.items():
                f = v.numpy().astype(np.float64).reshape(-1)
                got = np.concatenate([[f.sum(), np.abs(f).sum()], f[:4], f[-1:]])
                np.testing.assert_array_equal(got, d[f"{tag}/s{seed}/a{ai}/{k}"], err_msg=f"s{seed} a{ai} {k}")


def test_conv_halo_support_matrix_and_bad_arguments_without_gpu():
    """mzba_conv_halo(_ex)'s support checks and argument checks run before any HIP call: the 21x21 latent
    convs (gathered / action-bias form too), the 84x84 and 42x42 representation convs (two-block staging past
    W = 30 at Cin 256), Cout 128 only with all Cin channels staged at once, no gather past two envs per staged
    range (4x5), no action-bias table with a residual, null buffers."""
    import ctypes
    from mzba import _lib
    L = _lib.lib()
    sup = {(H, W, ci, co): (L.mzba_conv_halo_supported(H, W, ci, co, 3), L.mzba_conv_halo_ex_supported(H, W, ci, co, 3, 1))
           for H, W, ci, co in [(21, 21, 256, 256), (21, 21, 256, 128), (42, 42, 256, 256), (84, 84, 256, 256),
                                (84, 84, 128, 128), (84, 84, 128, 256), (42, 42, 256, 128), (84, 84, 64, 128),
                                (4, 5, 256, 256)]}
    assert sup == {(21, 21, 256, 256): (1, 1), (21, 21, 256, 128): (1, 0), (42, 42, 256, 256): (1, 0),
                   (84, 84, 256, 256): (1, 0), (84, 84, 128, 128): (1, 0), (84, 84, 128, 256): (1, 0),
                   (42, 42, 256, 128): (0, 0), (84, 84, 64, 128): (0, 0), (4, 5, 256, 256): (1, 0)}
    assert L.mzba_conv_halo_supported(21, 21, 256, 256, 1) == 0
    p = ctypes.c_void_p(64)
    n = 21 * 21 * 256
    # null input / weights / bias / output
    assert L.mzba_conv_halo_ex(None, n, None, 0, p, p, None, None, 0, None, p, 4, 21, 21, 256, 256, 1, None) == -1
    assert L.mzba_conv_halo_ex(p, n, None, 0, p, None, None, None, 0, None, p, 4, 21, 21, 256, 256, 1, None) == -1
    # action-bias table without actions, with a residual
    assert L.mzba_conv_halo_ex(p, n, None, 0, p, p, p, None, 3, None, p, 4, 21, 21, 256, 256, 1, None) == -1
    assert L.mzba_conv_halo_ex(p, n, None, 0, p, p, p, p, 3, p, p, 4, 21, 21, 256, 256, 1, None) == -1
    # gather where a staged range spans more than two envs; unsupported widths
    assert L.mzba_conv_halo_ex(p, 2 * 20 * 256, p, 20 * 256, p, p, None, None, 0, None, p, 4, 4, 5, 256, 256, 1,
                               None) == -2
    assert L.mzba_conv_halo_ex(p, 21 * 21 * 64, None, 0, p, p, None, None, 0, None, p, 4, 21, 21, 64, 256, 1, None) == -2
    assert L.mzba_conv_halo(p, p, p, None, p, 4, 42, 42, 256, 128, 1, None) == -2
    # the one-block bounds halo_geometry computes with the 16-row zero block: at Cin 256 one
    # 256-channel block up to W = 23 (so the gathered GA instance, which needs it, up to W = 23; past it the
    # plain conv stages two 128-channel blocks); at Cin 128 one block up to W = 183, and nothing past it
    assert L.mzba_conv_halo_ex_supported(23, 23, 256, 256, 3, 1) == 1
    assert L.mzba_conv_halo_ex_supported(24, 24, 256, 256, 3, 1) == 0
    assert L.mzba_conv_halo_supported(24, 24, 256, 256, 3) == 1
    assert L.mzba_conv_halo_supported(24, 24, 256, 128, 3) == 0  # Cout 128 needs one staged block
    assert L.mzba_conv_halo_supported(8, 183, 128, 128, 3) == 1
    assert L.mzba_conv_halo_supported(8, 184, 128, 128, 3) == 0
    assert L.mzba_conv_halo_supported(8, 183, 256, 256, 3) == 1
    assert L.mzba_conv_halo_supported(8, 184, 256, 256, 3) == 0


def test_learner_optimizer_param_groups_persist_and_lr_writes_reach_the_learner():
    """`for g in opt.param_groups: g["lr"] = x` must act like torch.optim.Adam's — one persistent group
    whose lr the next step() uses; the kernel's fixed hyperparameters refuse a change instead of ignoring it."""
    from mzba.agent import LearnerOptimizer

    class Ln:
        lr = 1e-3

    class Ag:
        _learner = Ln()
        cfg = {"learning_rate": 1e-3}

        def parameters(self):
            return iter([np.zeros(1)])

    opt = LearnerOptimizer(Ag())
    assert opt.param_groups is opt.param_groups
    for g in opt.param_groups:
        g["lr"] = 2.5e-4
    opt._sync_groups(Ag._learner)
    assert Ag._learner.lr == 2.5e-4
    opt.param_groups[0]["betas"] = [0.9, 0.999]  # a list equal to the constant is fine
    opt._sync_groups(Ag._learner)
    opt.param_groups[0]["weight_decay"] = 0.0
    with pytest.raises(NotImplementedError):
        opt._sync_groups(Ag._learner)
