"""Reference-format parameter sets for the three MuZero nets.

`state_dict_spec(model_cfg)` lists (key, shape) exactly as `MuZeroAgent.state_dict()`
orders them (src/networks.py:245-266; RepresentationNetwork :38-99, DynamicsNetwork
:103-167, PredictionNetwork :170-241), so a reference checkpoint's
`model_state_dict` (train_torch.py:620-621) loads unchanged.

`init_state_dict(model_cfg, seed)` is the documented synthetic initialiser used by
bench.py and the parity fixtures: the torch default distributions
(Conv2d/Linear: weight, bias ~ U(-1/sqrt(fan_in), +1/sqrt(fan_in)); BatchNorm:
gamma=1, beta=0, running_mean=0, running_var=1) drawn from
numpy.random.Generator(PCG64(seed)) in spec order, float32.
"""
from collections import OrderedDict

import numpy as np


def _conv_keys(p, cin, cout, k, bn):
    out = [(p + (".conv" if bn else "") + ".weight", (cout, cin, k, k)),
           (p + (".conv" if bn else "") + ".bias", (cout,))]
    if bn:
        out += _bn_keys(p + ".bn", cout)
    return out


def _bn_keys(p, c):
    return [(p + ".weight", (c,)), (p + ".bias", (c,)), (p + ".running_mean", (c,)),
            (p + ".running_var", (c,)), (p + ".num_batches_tracked", ())]


def _res_keys(p, c):
    return ([(p + ".conv1.weight", (c, c, 3, 3)), (p + ".conv1.bias", (c,))] + _bn_keys(p + ".bn1", c)
            + [(p + ".conv2.weight", (c, c, 3, 3)), (p + ".conv2.bias", (c,))] + _bn_keys(p + ".bn2", c))


def rep_layout(mcfg):
    """Module order of RepresentationNetwork.blocks (networks.py:46-92); avg-pool
    entries occupy ModuleList indices but hold no parameters."""
    n0, n1, n2 = mcfg["representation_network"]["num_res_blocks"]
    seq, i = [("conv", 0)], 1
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


def state_dict_spec(mcfg):
    c0, c1 = mcfg["latent_channels"]
    L = mcfg["state_history_length"]
    lr = mcfg["latent_resolution"]
    na = mcfg["dynamics_network"]["num_actions"]
    ns = mcfg["num_supports"]
    npol = mcfg["prediction_network"]["num_actions"]
    spec = []
    cin = 2 * L  # networks.py:248
    convs_seen = 0
    for kind, i in rep_layout(mcfg):
        p = f"rep_net.blocks.{i}"
        if kind == "conv":
            cout = c0 if convs_seen == 0 else c1
            spec += [(p + ".weight", (cout, cin, 3, 3)), (p + ".bias", (cout,))]
            cin = cout
            convs_seen += 1
        elif kind == "res":
            spec += _res_keys(p, cin)
    spec += _conv_keys("dyn_net.conv_block", c1 + na, c1, 3, True)
    for i in range(mcfg["dynamics_network"]["num_res_blocks"]):
        spec += _res_keys(f"dyn_net.res_blocks.{i}", c1)
    spec += _conv_keys("dyn_net.reward_head.0", c1, c1, 1, True)
    spec += [("dyn_net.reward_head.2.weight", (ns, c1 * lr[0] * lr[1])), ("dyn_net.reward_head.2.bias", (ns,))]
    for i in range(mcfg["prediction_network"]["num_res_blocks"]):
        spec += _res_keys(f"pred_net.res_blocks.{i}", c1)
    spec += _conv_keys("pred_net.policy_head.0", c1, c1 // 2, 3, True)
    spec += [("pred_net.policy_head.2.weight", (npol, (c1 // 2) * lr[0] * lr[1])), ("pred_net.policy_head.2.bias", (npol,))]
    spec += _conv_keys("pred_net.value_head.0", c1, c1 // 2, 1, True)
    spec += [("pred_net.value_head.2.weight", (ns, (c1 // 2) * lr[0] * lr[1])), ("pred_net.value_head.2.bias", (ns,))]
    return spec


def init_state_dict(mcfg, seed=0):
    g = np.random.Generator(np.random.PCG64(seed))
    sd = OrderedDict()
    spec = state_dict_spec(mcfg)
    shapes = dict(spec)
    for key, shape in spec:
        leaf = key.rsplit(".", 1)[1]
        if key.endswith("num_batches_tracked"):
            sd[key] = np.zeros((), dtype=np.int64)
        elif ".bn" in key or (".bn." in key):
            if leaf == "weight" or leaf == "running_var":
                sd[key] = np.ones(shape, dtype=np.float32)
            else:
                sd[key] = np.zeros(shape, dtype=np.float32)
        elif leaf == "weight":
            fan_in = int(np.prod(shape[1:]))
            bound = 1.0 / np.sqrt(fan_in)
            sd[key] = g.uniform(-bound, bound, size=shape).astype(np.float32)
        else:  # conv / linear bias: bound from the sibling weight's fan-in
            wshape = shapes[key[: -len("bias")] + "weight"]
            fan_in = int(np.prod(wshape[1:]))
            bound = 1.0 / np.sqrt(fan_in)
            sd[key] = g.uniform(-bound, bound, size=shape).astype(np.float32)
    return sd
