"""Drop-in module for the reference's `environment.parallel_breakout` (config.yaml:53-54
`environment_path`): resolves `BreakoutEnvironment` to the MI355X implementation."""
from abc import ABC, abstractmethod

from mzba.env import BreakoutEnvironment  # noqa: F401


class MuZeroEnvironment(ABC):
    """parallel_breakout.py:11-56 (interface only)."""

    @abstractmethod
    def reset(self):
        pass

    @abstractmethod
    def step(self, state, action):
        pass

    @abstractmethod
    def get_valid_actions(self, state):
        pass

    @property
    @abstractmethod
    def action_space_size(self):
        pass

    @property
    @abstractmethod
    def state_shape(self):
        pass


MuZeroEnvironment.register(BreakoutEnvironment)
