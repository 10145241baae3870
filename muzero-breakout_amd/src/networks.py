"""Drop-in module for the reference's `src.networks` (train_torch.py:86 loads
`get_class("src.networks", cfg["model"]["agent_name"])`)."""
from mzba.agent import MuZeroAgent  # noqa: F401
