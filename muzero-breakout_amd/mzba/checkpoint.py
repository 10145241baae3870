"""The reference's checkpoint format (train_torch.py:612-675).

`save_checkpoint` writes the dict `RLSystem._save_weights` writes (model_state_dict with the
reference keys, optimizer_state_dict, counters, replay_buffer lists), so the reference's
`_load_weights` reads it; `load_checkpoint` reads a reference checkpoint into this build's
agent (BN-folded packs rebuilt by `load_state_dict`) and device replay buffer. Files are read
with `torch.load(weights_only=True)`: tensors, lists, dicts and numbers only.
"""
import numpy as np
import torch

REPLAY_KEYS = ("past_actions_buffer", "future_actions_buffer", "state_buffer", "reward_buffer",
               "visit_counts_buffer", "value_buffer", "reward_sums", "length", "max_length", "bootstrapped_values")


def save_checkpoint(path, agent, replay=None, training_iteration=0, acting_step=0, iteration=0,
                    optimizer_state=None):
    """train_torch.py:612-637."""
    sd = {k: torch.from_numpy(np.array(v, copy=True)) for k, v in agent.state_dict().items()}  # keeps 0-d shapes
    torch.save({
        "model_state_dict": sd,
        "optimizer_state_dict": optimizer_state if optimizer_state is not None else {"state": {}, "param_groups": []},
        "training_iteration": training_iteration,
        "acting_step": acting_step,
        "iteration": iteration,
        "replay_buffer": replay.to_reference_lists() if replay is not None else
        {k: ([] if k not in ("length", "max_length") else 0) for k in REPLAY_KEYS},
    }, path)


def load_checkpoint(path, agent=None, replay=None):
    """train_torch.py:640-672: model weights into `agent`, replay lists into `replay`;
    returns the checkpoint dict (counters, optimizer state)."""
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    if agent is not None:
        agent.load_state_dict(ckpt["model_state_dict"])
    if replay is not None:
        replay.load_reference_lists(ckpt["replay_buffer"])
    return ckpt
