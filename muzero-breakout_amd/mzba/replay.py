"""Device replay buffer: drop-in for replay_buffer.py:ReplayBuffer.

The windows the reference builds in a Python triple loop (`save_observation_trajectory`,
replay_buffer.py:96-165) are built on the device (csrc/replay.hip) straight from the acting
loop's sink (`ingest_records`) or from host `ObservationTrajectory` objects
(`save_observation_trajectory`, same arithmetic). Storage is a FIFO ring of `max_length`
fixed-size rows in HBM (frames as u8 gray codes, 10 KB per window at 16x20); the getters
return device tensors with the reference's dtypes and shapes.
"""
import numpy as np
import torch

from . import _lib as L
from .env import gray_lut


class DeviceReplayBuffer:
    """ReplayBuffer(seq_len, K, max_length, discount, num_rewards_to_sum) (replay_buffer.py:76-92)."""

    def __init__(self, seq_len, K, max_length, discount, num_rewards_to_sum, height=16, width=20, device="cuda"):
        L.require_gpu()
        self.hist_seq_len, self.K, self.max_length = seq_len, K, max_length
        self.discount, self.num_rewards_to_sum = discount, num_rewards_to_sum
        self.H, self.W = height, width
        self.device = torch.device(device)
        cap, dev = max_length, self.device
        self._ring = {
            "past_actions": torch.zeros(cap, seq_len, dtype=torch.int64, device=dev),
            "future_actions": torch.zeros(cap, K, dtype=torch.int64, device=dev),
            "states": torch.zeros(cap, seq_len, height * width, dtype=torch.uint8, device=dev),
            "rewards": torch.zeros(cap, K, dtype=torch.float32, device=dev),
            "counts": torch.zeros(cap, K, 3, dtype=torch.float32, device=dev),
            "values": torch.zeros(cap, K, dtype=torch.float32, device=dev),
            "targets": torch.zeros(cap, K, dtype=torch.float32, device=dev),
            "reward_sum": torch.zeros(cap, dtype=torch.float32, device=dev),
        }
        self._lut = torch.from_numpy(gray_lut()).to(dev)
        self.start = 0      # ring slot of the oldest window
        self.length = 0     # windows stored (replay_buffer.py:87)
        self._dpow = {}

    def __len__(self):
        return self.length

    # -- ingest ------------------------------------------------------------------------
    def _powers(self, T):
        if T not in self._dpow:
            d = self.discount
            tab = [d ** k for k in range(T + 1)] + [d ** self.K]  # python double pow, as the reference
            self._dpow[T] = torch.tensor(np.array(tab, dtype=np.float64).astype(np.float32), device=self.device)
        return self._dpow[T]

    def ingest_records(self, rec, frame0, T, min_len=None):
        """Every trajectory of an acting-loop episode batch: rec = the loop's sink dict of
        (T_max, B, ...) device tensors (first T rows used), frame0 u8 [B][H*W] = g(s0) codes.
        Trajectories with length <= min_len (default K + 1, train_torch.py:224) are skipped;
        the rest are saved in env order, like the reference's loop over trajectories."""
        min_len = self.K + 1 if min_len is None else min_len
        B = rec["action"].shape[1]
        HW = self.H * self.W
        if rec.get("frame") is None:
            raise ValueError("ingest_records needs the loop's recorded frames (record_frames=True)")
        dev = self.device
        lens = torch.empty(B, dtype=torch.int32, device=dev)
        rsum = torch.empty(B, dtype=torch.float32, device=dev)
        offs = torch.empty(B + 1, dtype=torch.int32, device=dev)
        args = (L.ptr(rec["action"]), L.ptr(rec["reward"]), L.ptr(rec["mask"]), L.ptr(rec["counts"]),
                L.ptr(rec["values"]), L.ptr(rec["frame"]), L.ptr(frame0), T, B, HW)
        L.call("mzba_replay_plan", *args, self.K, min_len, L.ptr(lens), L.ptr(rsum), L.ptr(offs), L.stream())
        n = int(offs[B].item())
        self._write(args, lens, rsum, offs, n, T)
        return n

    def _write(self, args, lens, rsum, offs, n, T):
        cap = self.max_length
        head = (self.start + self.length) % cap
        g = self._ring
        L.call("mzba_replay_write", *args, L.ptr(lens), L.ptr(rsum), L.ptr(offs), n, L.ptr(g["past_actions"]),
               L.ptr(g["future_actions"]), L.ptr(g["states"]), L.ptr(g["rewards"]), L.ptr(g["counts"]),
               L.ptr(g["values"]), L.ptr(g["targets"]), L.ptr(g["reward_sum"]), cap, head, self.K,
               self.hist_seq_len, L.ptr(self._powers(T)), L.stream())
        total = self.length + n
        self.length = min(total, cap)
        self.start = (self.start + total - self.length) % cap

    def save_observation_trajectory(self, observation_trajectory):
        """replay_buffer.py:96-165 for one host trajectory (padded as _pad_initial_state builds it)."""
        t = observation_trajectory
        h, Lr = self.hist_seq_len, t.length
        if Lr == 0:
            return
        inv = {float(v): c for c, v in reversed(list(enumerate(gray_lut())))}

        def codes(img):
            a = np.asarray(img.cpu() if torch.is_tensor(img) else img, dtype=np.float32).reshape(-1)
            try:
                return np.array([inv[float(x)] for x in a], dtype=np.uint8)
            except KeyError as e:
                raise ValueError(f"state value {e} is not a convert_to_grayscale output") from None

        dev = self.device
        T = Lr
        tensor = lambda x, dt: torch.as_tensor(np.ascontiguousarray(x), dtype=dt, device=dev)  # noqa: E731
        rec = {
            "action": tensor(np.array([int(a) for a in t.actions[h:]], np.uint8).reshape(T, 1), torch.uint8),
            "reward": tensor(np.array([float(r) for r in t.rewards[h:]], np.float32).reshape(T, 1), torch.float32),
            "mask": torch.ones(T, 1, dtype=torch.uint8, device=dev),
            "counts": tensor(np.stack([np.asarray(c.cpu() if torch.is_tensor(c) else c) for c in
                                       t.visit_counts[h:]]).astype(np.int64).reshape(T, 1, 3), torch.int64),
            "values": tensor(np.array([float(v) for v in t.values[h:]], np.float32).reshape(T, 1), torch.float32),
            "frame": tensor(np.stack([codes(s) for s in t.states[h - 1:]]).reshape(T, 1, -1), torch.uint8),
        }
        frame0 = tensor(codes(t.states[0]).reshape(1, -1), torch.uint8)
        self.ingest_records(rec, frame0, T, min_len=-1)

    # -- getters (replay_buffer.py:167-225) --------------------------------------------------
    def _slots(self, batch_idxs):
        idx = torch.as_tensor(batch_idxs, device=self.device).to(torch.int64)
        if idx.numel():
            lo, hi = torch.stack([idx.min(), idx.max()]).tolist()
            if lo < 0 or hi >= self.length:
                raise IndexError("replay index out of range")
        return (idx + self.start) % self.max_length

    def get_batched_past_actions(self, batch_idxs):
        return self._ring["past_actions"][self._slots(batch_idxs)]

    def get_batched_future_actions(self, batch_idxs):
        return self._ring["future_actions"][self._slots(batch_idxs)]

    def get_batched_states(self, batch_idxs):
        """[batch, hist, 1, H, W] f32 grayscale (the stacked (1, H, W) frames)."""
        slots = self._slots(batch_idxs).to(torch.int32)
        n = slots.numel()
        out = torch.empty(n, self.hist_seq_len, 1, self.H, self.W, dtype=torch.float32, device=self.device)
        L.call("mzba_replay_states", L.ptr(self._ring["states"]), L.ptr(slots), n, L.ptr(self._lut), L.ptr(out),
               self.hist_seq_len, self.H * self.W, L.stream())
        return out

    def get_batched_rewards(self, batch_idxs):
        return self._ring["rewards"][self._slots(batch_idxs)]

    def get_batched_visit_counts(self, batch_idxs):
        return self._ring["counts"][self._slots(batch_idxs)]

    def get_batched_values(self, batch_idxs):
        """The bootstrapped n-step value targets (replay_buffer.py:209-214)."""
        return self._ring["targets"][self._slots(batch_idxs)]

    def get_values(self, batch_idxs):
        """value_buffer rows (the searched root values) — kept for inspection."""
        return self._ring["values"][self._slots(batch_idxs)]

    def get_reward_sums(self):
        """Reward sums of the newest `num_rewards_to_sum` windows (replay_buffer.py:221-225)."""
        n = min(self.num_rewards_to_sum, self.length)
        idx = torch.arange(self.length - n, self.length, device=self.device)
        return [float(x) for x in self._ring["reward_sum"][self._slots(idx)].cpu()]

    def empty_buffer(self):
        self.start = self.length = 0

    # -- the reference's list layout (checkpoint replay_buffer, train_torch.py:624-635) ----
    def to_reference_lists(self):
        idx = torch.arange(self.length, device=self.device)
        cpu = lambda t: list(t.cpu().unbind(0)) if self.length else []  # noqa: E731
        sl = self._slots(idx) if self.length else idx
        return {
            "past_actions_buffer": cpu(self._ring["past_actions"][sl]),
            "future_actions_buffer": cpu(self._ring["future_actions"][sl]),
            "state_buffer": cpu(self.get_batched_states(idx)) if self.length else [],
            "reward_buffer": cpu(self._ring["rewards"][sl]),
            "visit_counts_buffer": cpu(self._ring["counts"][sl]),
            "value_buffer": cpu(self._ring["values"][sl]),
            "reward_sums": [float(x) for x in self._ring["reward_sum"][sl].cpu()],
            "length": self.length,
            "max_length": self.max_length,
            "bootstrapped_values": cpu(self._ring["targets"][sl]),
        }

    def load_reference_lists(self, d):
        """Replace the contents with a reference replay_buffer dict (oldest first)."""
        n = int(d["length"])
        if n > self.max_length:
            raise ValueError(f"checkpoint holds {n} windows, buffer max_length is {self.max_length}")
        self.empty_buffer()
        if n == 0:
            return
        lut = gray_lut()
        vals, first = np.unique(lut, return_index=True)
        st = np.stack([np.asarray(s, np.float32) for s in d["state_buffer"][:n]]).reshape(n, self.hist_seq_len, -1)
        pos = np.searchsorted(vals, st).clip(0, len(vals) - 1)
        if not np.array_equal(vals[pos], st):
            raise ValueError("state_buffer holds values that are not convert_to_grayscale outputs")
        g, dev = self._ring, self.device
        put = lambda key, rows, dt: g[key][:n].copy_(torch.as_tensor(np.stack([np.asarray(x) for x in rows]),  # noqa: E731
                                                                  dtype=dt).to(dev))
        g["states"][:n].copy_(torch.from_numpy(first[pos].astype(np.uint8)).to(dev))
        put("past_actions", d["past_actions_buffer"][:n], torch.int64)
        put("future_actions", d["future_actions_buffer"][:n], torch.int64)
        put("rewards", d["reward_buffer"][:n], torch.float32)
        put("counts", d["visit_counts_buffer"][:n], torch.float32)
        put("values", d["value_buffer"][:n], torch.float32)
        put("targets", d["bootstrapped_values"][:n], torch.float32)
        g["reward_sum"][:n].copy_(torch.tensor(np.asarray(d["reward_sums"][:n], np.float32)).to(dev))
        self.start, self.length = 0, n
