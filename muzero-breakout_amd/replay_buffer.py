"""Drop-in module for the reference's `replay_buffer` (replay_buffer.py): the trajectory record
type of the acting loop's sink and the replay buffer, whose window slicing and n-step value
targets run on the device (mzba/replay.py, csrc/replay.hip)."""
from mzba.acting import ObservationTrajectory  # noqa: F401
from mzba.replay import DeviceReplayBuffer as ReplayBuffer  # noqa: F401
