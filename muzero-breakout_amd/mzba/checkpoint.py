"""The reference's checkpoint format (train_torch.py:612-675).

`save_checkpoint` writes the dict `RLSystem._save_weights` writes (model_state_dict with the
reference keys, optimizer_state_dict, counters, replay_buffer lists), so the reference's
`_load_weights` reads it — including `optimizer.load_state_dict`, which needs one Adam param group
listing every parameter of `MuZeroAgent.parameters()` (networks.py:268): a learner's own Adam state
when one is given, else a fresh Adam state of that shape. `load_checkpoint` reads a reference
checkpoint into this build's agent (BN-folded packs rebuilt by `load_state_dict`), learner (weights
and Adam moments) and device replay buffer. Files are read with `torch.load(weights_only=True)`:
tensors, lists, dicts and numbers only.
"""
import numpy as np
import torch

from .weights import state_dict_spec

REPLAY_KEYS = ("past_actions_buffer", "future_actions_buffer", "state_buffer", "reward_buffer",
               "visit_counts_buffer", "value_buffer", "reward_sums", "length", "max_length", "bootstrapped_values")
WEIGHT_DECAY = 1e-4  # networks.py:268


def n_parameters(mcfg):
    """Entries of MuZeroAgent.parameters(): every state_dict key but the BN buffers."""
    return sum(1 for k, _ in state_dict_spec(mcfg)
               if not k.endswith(("running_mean", "running_var", "num_batches_tracked")))


def fresh_optimizer_state(mcfg, lr=None):
    """`torch.optim.Adam(mu_zero.parameters(), lr, weight_decay=1e-4).state_dict()` before any step."""
    lr = float(mcfg["learning_rate"] if lr is None else lr)
    group = dict(torch.optim.Adam([torch.zeros(1)], lr=lr, weight_decay=WEIGHT_DECAY).state_dict()["param_groups"][0])
    group["params"] = list(range(n_parameters(mcfg)))
    return {"state": {}, "param_groups": [group]}


def save_checkpoint(path, agent, replay=None, training_iteration=0, acting_step=0, iteration=0,
                    optimizer_state=None, learner=None):
    """train_torch.py:612-637. The optimizer state is, in order of preference: `optimizer_state`,
    `learner.optimizer_state_dict()`, a fresh Adam state for the agent's parameters."""
    sd = {k: (v.detach().clone() if torch.is_tensor(v) else torch.from_numpy(np.array(v, copy=True)))
          for k, v in agent.state_dict().items()}  # own copies; keeps 0-d shapes
    if optimizer_state is None:
        optimizer_state = learner.optimizer_state_dict() if learner is not None else fresh_optimizer_state(agent.cfg)
    torch.save({
        "model_state_dict": sd,
        "optimizer_state_dict": optimizer_state,
        "training_iteration": training_iteration,
        "acting_step": acting_step,
        "iteration": iteration,
        "replay_buffer": replay.to_reference_lists() if replay is not None else
        {k: ([] if k not in ("length", "max_length") else 0) for k in REPLAY_KEYS},
    }, path)


def load_checkpoint(path, agent=None, replay=None, learner=None):
    """train_torch.py:640-672: model weights into `agent` (and `learner`, whose Adam moments come from
    the optimizer_state_dict), replay lists into `replay`; returns the checkpoint dict."""
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    if agent is not None:
        agent.load_state_dict(ckpt["model_state_dict"])
    if learner is not None:
        learner.load_state_dict(ckpt["model_state_dict"])
        learner.load_optimizer_state_dict(ckpt["optimizer_state_dict"])
    if replay is not None:
        replay.load_reference_lists(ckpt["replay_buffer"])
    return ckpt
