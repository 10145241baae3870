"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

Restatement of the reference replay buffer (`replay_buffer.py:76-232`):
`ReplayBuffer.save_observation_trajectory` (window slicing, n-step value targets, FIFO
eviction) and the `get_batched_*` getters, in numpy with the reference's f32 arithmetic.

A trajectory is the reference's padded `ObservationTrajectory` (`train_torch.py:313-332`):
32 padding actions 0, 31 padding frames g(s0), 32 padding rewards / values 0 and visit
counts zeros(3), then `length` real records. Quirks kept: the value target bootstraps
`td_steps = 10` ahead but scales by `discount ** K` (`replay_buffer.py:137-145`); the states
list has one padding entry fewer than the actions (`train_torch.py:324-325`), so a window's
frames are shifted by one against its past actions.
"""
import numpy as np

f32 = np.float32


def value_targets(values, rewards, state_start, K, L, discount, hist=32, td_steps=10):
    """replay_buffer.py:137-151 for one window: K targets, f32 op order of the torch code
    (`v * discount**K` then `+= discount**k * r`, python floats rounded to f32)."""
    max_length = hist + L
    out = np.zeros(K, dtype=np.float32)
    bootstrap_idx = state_start + td_steps
    for i, cur in enumerate(range(state_start, state_start + K)):
        if bootstrap_idx < max_length:
            t = f32(values[bootstrap_idx] * f32(discount ** K))
            for k, r in enumerate(rewards[cur:bootstrap_idx]):
                t = f32(t + f32(f32(discount ** k) * r))
        else:
            t = None  # python 0.0 + the first f32 term is that term exactly
            for k, r in enumerate(rewards[cur:max_length]):
                term = f32(f32(discount ** k) * r)
                t = term if t is None else f32(t + term)
        out[i] = t
        bootstrap_idx += 1
    return out


class ReplayOracle:
    """ReplayBuffer(seq_len, K, max_length, discount, num_rewards_to_sum) on numpy records."""

    def __init__(self, seq_len, K, max_length, discount, num_rewards_to_sum):
        self.hist, self.K, self.max_length = seq_len, K, max_length
        self.discount, self.num_rewards_to_sum = discount, num_rewards_to_sum
        self.rows = []  # FIFO of dicts (one per window)

    def save(self, actions, frames, frame0, rewards, counts, values):
        """One trajectory of `L` real records: actions i64[L], frames [L][H][W] (grayscale f32),
        frame0 [H][W] (g(s0)), rewards f32[L], counts [L][3], values f32[L]
        (replay_buffer.py:96-165 on the padded lists)."""
        h, K = self.hist, self.K
        L = len(actions)
        acts = np.concatenate([np.zeros(h, np.int64), np.asarray(actions, np.int64)])
        states = np.concatenate([np.repeat(frame0[None], h - 1, 0), np.asarray(frames, np.float32)])
        rews = np.concatenate([np.zeros(h, np.float32), np.asarray(rewards, np.float32)])
        vcs = np.concatenate([np.zeros((h, 3), np.float32), np.asarray(counts, np.float32)])
        vals = np.concatenate([np.zeros(h, np.float32), np.asarray(values, np.float32)])
        rsum = f32(0)
        for r in np.asarray(rewards, np.float32):
            rsum = f32(rsum + r)  # ObservationTrajectory.reward_sum (replay_buffer.py:34)
        for state in range(L - K + 1):
            ss = state + h
            ts = ss - h
            self.rows.append({
                "past_actions": acts[ts:ss].copy(),
                "future_actions": acts[ss:ss + K].copy(),
                "states": states[ts:ss].copy(),
                "reward_sum": rsum,
                "rewards": rews[ss:ss + K].copy(),
                "visit_counts": vcs[ss:ss + K].copy(),
                "values": vals[ss:ss + K].copy(),
                "targets": value_targets(vals, rews, ss, K, L, self.discount, h),
            })
            if len(self.rows) > self.max_length:  # :154-165
                self.rows.pop(0)

    def __len__(self):
        return len(self.rows)

    def batched(self, key, idxs):
        return np.stack([self.rows[i][key] for i in idxs])

    def reward_sums(self):
        """get_reward_sums (:221-225)."""
        return np.array([r["reward_sum"] for r in self.rows[-self.num_rewards_to_sum:]], dtype=np.float32)
