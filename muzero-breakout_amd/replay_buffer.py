"""Drop-in module for the reference's `replay_buffer` record type (the acting loop's sink).
`ReplayBuffer` itself (replay_buffer.py:76-232) is a SURVEY §8(f) "next" row."""
from mzba.acting import ObservationTrajectory  # noqa: F401
