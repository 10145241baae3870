"""Drop-in module for the reference's `src.mcts` (train_torch.py:90 loads
`get_class("src.mcts", cfg["search"]["mcts_name"])`)."""
from mzba.search import MCTSSearchVec  # noqa: F401
