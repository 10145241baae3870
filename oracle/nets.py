"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

numpy (f32 by default) restatement of the reference networks
(`src/networks.py`) in eval mode, driven by a reference-format `state_dict`
(same keys and shapes as `MuZeroAgent.state_dict()`), and of the scalar decode
(`utils.py:ScalarTransforms`). Conv = im2col + matmul; BN eval = x*alpha + beta
with alpha = w/sqrt(var+eps), beta = b - mean*alpha (torch CPU eval BN form).
Pinned against reference outputs in tests/golden/nets_*.npz.
"""
import numpy as np

BN_EPS = 1e-5


def _conv(x, w, b, pad):
    """x (B,C,H,W), w (O,C,k,k) -> (B,O,H,W); stride 1, zero padding."""
    B, C, H, W = x.shape
    O, _, k, _ = w.shape
    dt = x.dtype
    if pad:
        xp = np.zeros((B, C, H + 2 * pad, W + 2 * pad), dtype=dt)
        xp[:, :, pad:pad + H, pad:pad + W] = x
    else:
        xp = x
    cols = np.empty((B, H, W, C, k, k), dtype=dt)
    for dy in range(k):
        for dx in range(k):
            cols[:, :, :, :, dy, dx] = xp[:, :, dy:dy + H, dx:dx + W].transpose(0, 2, 3, 1)
    cols = cols.reshape(B * H * W, C * k * k)
    out = cols @ w.reshape(O, C * k * k).astype(dt).T
    out = out.reshape(B, H, W, O).transpose(0, 3, 1, 2)
    if b is not None:
        out = out + b.astype(dt)[None, :, None, None]
    return np.ascontiguousarray(out)


def _bn(x, sd, p):
    w = sd[p + ".weight"].astype(x.dtype)
    b = sd[p + ".bias"].astype(x.dtype)
    m = sd[p + ".running_mean"].astype(x.dtype)
    v = sd[p + ".running_var"].astype(x.dtype)
    alpha = w / np.sqrt(v + x.dtype.type(BN_EPS))
    beta = b - m * alpha
    return x * alpha[None, :, None, None] + beta[None, :, None, None]


def _relu(x):
    return np.maximum(x, x.dtype.type(0))


def _resblock(x, sd, p):
    """networks.py:19-35: relu(bn2(conv2(relu(bn1(conv1(x))))) + x)."""
    x1 = _relu(_bn(_conv(x, sd[p + ".conv1.weight"], sd[p + ".conv1.bias"], 1), sd, p + ".bn1"))
    x2 = _bn(_conv(x1, sd[p + ".conv2.weight"], sd[p + ".conv2.bias"], 1), sd, p + ".bn2")
    return _relu(x2 + x)


def _convblock(x, sd, p, pad):
    """networks.py:7-17: relu(bn(conv(x)))."""
    w = sd[p + ".conv.weight"]
    return _relu(_bn(_conv(x, w, sd[p + ".conv.bias"], pad), sd, p + ".bn"))


def _avgpool2(x):
    B, C, H, W = x.shape
    x = x[:, :, : H // 2 * 2, : W // 2 * 2]
    return x.reshape(B, C, H // 2, 2, W // 2, 2).mean(axis=(3, 5), dtype=x.dtype)


def rep_layout(mcfg):
    """Module order of RepresentationNetwork.blocks (networks.py:46-92)."""
    n0, n1, n2 = mcfg["representation_network"]["num_res_blocks"]
    seq = [("conv", 0)]
    i = 1
    for _ in range(n0):
        seq.append(("res", i)); i += 1
    seq.append(("conv", i)); i += 1
    for _ in range(n1):
        seq.append(("res", i)); i += 1
    seq.append(("pool", i)); i += 1
    for _ in range(n2):
        seq.append(("res", i)); i += 1
    seq.append(("pool", i)); i += 1
    return seq


def representation(x, sd, mcfg):
    """networks.py:94-99."""
    for kind, i in rep_layout(mcfg):
        p = f"rep_net.blocks.{i}"
        if kind == "conv":
            x = _conv(x, sd[p + ".weight"], sd[p + ".bias"], 1)
        elif kind == "res":
            x = _resblock(x, sd, p)
        else:
            x = _avgpool2(x)
    return x


def scale_state(h):
    """networks.py:314-328: per-env min-max."""
    B = h.shape[0]
    flat = h.reshape(B, -1)
    mn = flat.min(axis=1).reshape(B, 1, 1, 1)
    mx = flat.max(axis=1).reshape(B, 1, 1, 1)
    return (h - mn) / (mx - mn + h.dtype.type(1e-8))


def dynamics(h, a_planes, sd, mcfg):
    """networks.py:151-167 (+ hidden_state_transition :282-298 incl. scaling)."""
    x = np.concatenate([h, a_planes.astype(h.dtype)], axis=1)
    x = _convblock(x, sd, "dyn_net.conv_block", 1)
    for i in range(mcfg["dynamics_network"]["num_res_blocks"]):
        x = _resblock(x, sd, f"dyn_net.res_blocks.{i}")
    r = _convblock(x, sd, "dyn_net.reward_head.0", 0)
    r = r.reshape(r.shape[0], -1) @ sd["dyn_net.reward_head.2.weight"].astype(h.dtype).T + sd["dyn_net.reward_head.2.bias"].astype(h.dtype)
    return scale_state(x), r


def prediction(h, sd, mcfg):
    """networks.py:225-241: (policy logits, value logits)."""
    x = h
    for i in range(mcfg["prediction_network"]["num_res_blocks"]):
        x = _resblock(x, sd, f"pred_net.res_blocks.{i}")
    p = _convblock(x, sd, "pred_net.policy_head.0", 1)
    p = p.reshape(p.shape[0], -1) @ sd["pred_net.policy_head.2.weight"].astype(h.dtype).T + sd["pred_net.policy_head.2.bias"].astype(h.dtype)
    v = _convblock(x, sd, "pred_net.value_head.0", 0)
    v = v.reshape(v.shape[0], -1) @ sd["pred_net.value_head.2.weight"].astype(h.dtype).T + sd["pred_net.value_head.2.bias"].astype(h.dtype)
    return p, v


def create_hidden_state_root(x, sd, mcfg):
    """networks.py:271-280."""
    return scale_state(representation(x, sd, mcfg))


def encode_action_planes(actions, latent_res, n_actions=3, dtype=np.float32):
    """mcts.py:252-268: one-hot planes tiled over the latent grid."""
    B = actions.shape[0]
    oh = np.zeros((B, n_actions), dtype=dtype)
    oh[np.arange(B), actions] = 1
    return np.broadcast_to(oh[:, :, None, None], (B, n_actions, latent_res[0], latent_res[1])).copy()


def softmax(x, axis=-1):
    m = x.max(axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=axis, keepdims=True)


def inverted_softmax_expectation(logits, smin=-5.0, smax=5.0):
    """utils.py:74-81 + :26-28: sign(x)*((|x|+0.999)^2-1), x = E_softmax[supports]."""
    n = logits.shape[-1]
    dt = logits.dtype
    supports = np.linspace(smin, smax, n).astype(dt)
    p = softmax(logits)
    x = (p * supports).sum(axis=-1)
    t = np.abs(x) + dt.type(1 - 0.001)
    return (np.sign(x) * (t * t - dt.type(1))).astype(dt)
