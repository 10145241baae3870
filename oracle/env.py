"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

numpy restatement of the reference Breakout environment
(`environment/parallel_breakout.py`), op for op, used as the checker for the HIP
env kernels and as the CPU baseline ("port"). Pinned against fixtures generated
from the reference itself (tests/golden/make_golden.py -> env_*.npz).
"""
import numpy as np

from . import rng as R

CH_PADDLE, CH_BALL, CH_BRICKS = 0, 1, 2  # parallel_breakout.py:88-90


class BreakoutEnvOracle:
    """Mirrors BreakoutEnvironment (parallel_breakout.py:59-254).

    Geometry is hard-coded by the reference (parallel_breakout.py:76-79): H=16, W=20,
    3 brick rows; `height`/`width` may be overridden after construction (84x84 case).
    """

    def __init__(self, cfg, paddle_width=6):
        self.height = 16
        self.width = 20
        self.paddle_width = paddle_width
        self.brick_rows = 3
        self.batch = cfg["n_parallel"]
        self.paddle_hit_reward = np.float32(cfg["paddle_hit_reward"])
        self.brick_hit_reward = np.float32(cfg["brick_hit_reward"])
        self.game_lost_reward = np.float32(cfg["game_lost_reward"])
        self.game_won_reward = np.float32(cfg["game_won_reward"])
        self.action_space_size = 3
        self.ball_dx = None
        self.ball_dy = None

    # -- reset ------------------------------------------------------------
    def reset_params(self, seed, episode, env_offset=0):
        """Draw reset randomness from the keyed stream (replaces the torch.randint
        calls at parallel_breakout.py:116,126,127,136)."""
        B, W, H, pw = self.batch, self.width, self.height, self.paddle_width
        env = np.arange(B, dtype=np.int64) + env_offset
        low = -6
        high = W - pw - (W // 2 - pw // 2 - 1)  # :115
        off = low + R.randbelow(env, R.STREAM_RESET, episode, 0, seed, high - low)
        col = 1 + R.randbelow(env, R.STREAM_RESET, episode, 1, seed, W - 2)
        row = -3 + R.randbelow(env, R.STREAM_RESET, episode, 2, seed, 2)
        dx = np.where(R.randbelow(env, R.STREAM_RESET, episode, 3, seed, 2) == 0, -1, 1)
        return off.astype(np.int64), col.astype(np.int64), row.astype(np.int64), dx.astype(np.int64)

    def reset(self, params):
        """parallel_breakout.py:107-139 with explicit draws (offset, ball col,
        ball row offset in {-3,-2}, dx)."""
        off, col, row, dx = params
        B, H, W, pw = self.batch, self.height, self.width, self.paddle_width
        state = np.zeros((B, 3, H, W), dtype=np.float32)
        paddle_pos = W // 2 - pw // 2 + off  # :120
        b = np.arange(B)[:, None]
        state[b, CH_PADDLE, H - 1, paddle_pos[:, None] + np.arange(pw)[None, :]] = 1  # :123
        state[np.arange(B), CH_BALL, (row % H), col] = 1  # :128 (negative row indexes from the bottom)
        state[:, CH_BRICKS, : self.brick_rows, :] = 1  # :131
        self.ball_dx = dx.astype(np.int64).copy()  # :136
        self.ball_dy = np.full(B, -1.0, dtype=np.float32)  # :137
        return state, 0

    # -- valid actions -----------------------------------------------------
    def get_valid_actions(self, state, paddle_pos_new):
        """parallel_breakout.py:141-155."""
        valid = np.ones((self.batch, self.action_space_size), dtype=np.float32)
        valid[paddle_pos_new == 0, 0] = 0
        valid[paddle_pos_new + self.paddle_width >= self.width, -1] = 0
        return valid

    # -- step --------------------------------------------------------------
    def step(self, state, action, done_mask):
        """parallel_breakout.py:158-254, op for op. `done_mask` (bool ndarray) is
        mutated in place and returned, like the reference."""
        H, W, pw = self.height, self.width, self.paddle_width
        B = self.batch
        next_state = state.copy()
        reward = np.zeros(B, dtype=np.float32)

        row = state[:, CH_PADDLE, H - 1, :]
        paddle_pos = np.argmax(row, axis=1)  # :177 first max
        delta = np.where(action == 0, -1, np.where(action == 2, 1, 0))
        paddle_pos_new = np.clip(paddle_pos + delta, 0, W - pw)  # :178-179
        bidx = np.arange(B)[:, None]
        next_state[:, CH_PADDLE, H - 1, :] = 0  # :183
        paddle_positions = paddle_pos_new[:, None] + np.arange(pw)[None, :]
        next_state[bidx, CH_PADDLE, H - 1, paddle_positions] = 1  # :186

        bb, by, bx = np.nonzero(state[:, CH_BALL] == 1)  # :189
        if bb.shape[0] != B or not np.array_equal(bb, np.arange(B)):
            raise IndexError("each env must hold exactly one ball")
        ball_x = bx.astype(np.float32)
        ball_y = by.astype(np.float32)

        dx = self.ball_dx
        wall = np.logical_or(ball_x + dx < 0, ball_x + dx >= W)  # :195
        dx = np.where(wall, -dx, dx)  # :196
        dy = self.ball_dy.copy()
        new_y = (ball_y + dy).astype(np.float32)  # :198
        new_x = (ball_x + dx).astype(np.float32)  # :199

        missed = new_y >= H  # :202
        reward[missed] = self.game_lost_reward  # :203
        done_mask |= missed  # :204
        next_state[done_mask, CH_BRICKS] = 0  # :205
        next_state[done_mask, CH_PADDLE] = 0  # :206
        dx = dx.copy()
        dx[done_mask] = 0  # :207
        dy[done_mask] = 0  # :208
        new_y[missed] = 0  # :209

        ceil = new_y < 0  # :213
        dy[ceil] *= np.float32(-1)
        ceil2 = new_y < 0  # :214 (re-evaluated; same mask)
        new_y[ceil2] = ball_y[ceil2]

        old_dy = dy.copy()  # :217
        new_x_br = (new_x - np.mod(new_x, np.float32(2))).astype(np.float32)  # :218 (torch % == floor-mod)
        yi = new_y.astype(np.int64)  # .int() truncation; values are exact ints
        xbi = new_x_br.astype(np.int64)
        b = np.arange(B)
        brick = next_state[b, CH_BRICKS, yi % H, xbi % W] == 1  # :219
        dy = np.where(brick, -old_dy, dy)  # :220
        next_state[b, CH_BRICKS, yi % H, xbi % W] = 0  # :221
        next_state[b, CH_BRICKS, yi % H, (xbi + 1) % W] = 0  # :222
        new_y = np.where(brick, (ball_y - old_dy).astype(np.float32), new_y).astype(np.float32)  # :224
        reward[brick] += self.brick_hit_reward  # :226

        prow = new_y == (H - 1)  # :229
        pmask = np.zeros((B, W), dtype=np.float32)
        pmask[bidx, paddle_positions] = 1  # :231-232
        hits = prow & (pmask[b, new_x.astype(np.int64) % W].astype(np.int64) != 0)  # :234
        dy = np.where(hits, -dy, dy)  # :235
        reward[hits] += self.paddle_hit_reward  # :239

        next_state[:, CH_BALL] = 0  # :242
        next_state[b, CH_BALL, new_y.astype(np.int64) % H, new_x.astype(np.int64) % W] = 1  # :243 (row -1 wraps)

        finished = ~next_state[:, CH_BRICKS].any(axis=(1, 2))  # :246
        done_mask |= finished  # :247
        next_state[done_mask, CH_BRICKS] = 0  # :248
        next_state[done_mask, CH_PADDLE] = 0  # :249
        reward[finished ^ missed] += self.game_won_reward  # :250

        self.ball_dx = dx
        self.ball_dy = dy.astype(np.float32)
        valid = self.get_valid_actions(next_state, paddle_pos_new)  # :252
        return next_state, reward, done_mask, valid


def convert_to_grayscale(state):
    """train_torch.py:334-358: clamp((0.3*paddle + 1.0*ball) + 0.6*bricks, 0, 1)."""
    paddle = state[:, 0] * np.float32(0.3)
    ball = state[:, 1] * np.float32(1.0)
    bricks = state[:, 2] * np.float32(0.6)
    g = (paddle + ball) + bricks
    return np.clip(g, 0, 1).astype(np.float32)[:, None]
