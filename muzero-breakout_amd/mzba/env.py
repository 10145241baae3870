"""Breakout environment on the MI355X path (mirror of
environment/parallel_breakout.py:BreakoutEnvironment).

`BreakoutEnvironment` keeps the reference's plane representation and API:
reset() -> (state f32 (B,3,H,W), 0); step(state, action, done_mask) ->
(next_state, reward, done_mask (the SAME tensor, mutated in place), valid_actions).
Computation runs in the HIP kernels; inputs on the CPU are moved to the device
and results are returned on the caller's device. Random draws come from the keyed
Philox stream (seed, global env, episode) instead of torch's global generator.

`CompactBreakout` is the acting loop's representation (SoA scalars + brick bitmask,
uint8 gray frames rendered in the same kernel); same rules, same outputs.
"""
import ctypes

import numpy as np
import torch

from . import _lib as L


class BreakoutEnvironment:
    def __init__(self, cfg, width=10, height=15, paddle_width=6, brick_rows=3, device="cuda", seed=0, env_offset=0,
                 state_device="cpu"):
        """`device`: where the kernels run; `state_device`: where reset() returns the state — the CPU,
        like the reference's env (parallel_breakout.py:80 `self.device = "cpu"`), so the reference's
        `_prepare_mcts_input` can concatenate it with its CPU action planes (train_torch.py:271-276).
        step() returns its outputs on the device of the state it is given."""
        L.require_gpu()
        self.state_device = torch.device(state_device)
        self.height = 16  # parallel_breakout.py:76-79 (hard-coded by the reference)
        self.width = 20
        self.paddle_width = paddle_width
        self.brick_rows = 3
        self.device = torch.device(device)
        self.batch = cfg["n_parallel"]
        self.paddle_hit_reward = cfg["paddle_hit_reward"]
        self.brick_hit_reward = cfg["brick_hit_reward"]
        self.game_lost_reward = cfg["game_lost_reward"]
        self.game_won_reward = cfg["game_won_reward"]
        self.CHANNEL_PADDLE, self.CHANNEL_BALL, self.CHANNEL_BRICKS = 0, 1, 2
        self._action_space_size = 3
        self.ball_dx = 1
        self.ball_dy = -1
        self.seed = seed
        self.env_offset = env_offset
        self.episode = 0

    @property
    def action_space_size(self):
        return self._action_space_size

    @property
    def state_shape(self):
        return (self.batch, 3, self.height, self.width)

    def reset(self, params=None):
        """parallel_breakout.py:107-139. `params` (optional int32 (4,B): paddle offset,
        ball col, ball row offset, dx) replaces the random draws."""
        B, H, W = self.batch, self.height, self.width
        state = torch.empty(B, 3, H, W, dtype=torch.float32, device=self.device)
        self.ball_dx = torch.empty(B, dtype=torch.int64, device=self.device)
        self.ball_dy = torch.empty(B, dtype=torch.float32, device=self.device)
        pr = None
        if params is not None:
            pr = torch.as_tensor(np.asarray(params, dtype=np.int32), device=self.device).contiguous()
        L.ops().env_reset_(state, self.ball_dx, self.ball_dy, self.paddle_width, self.brick_rows, self.seed,
                           self.episode, self.env_offset, pr)
        self.episode += 1
        return state.to(self.state_device), 0

    def get_valid_actions(self, state, paddle_pos_new):
        """parallel_breakout.py:141-155."""
        valid = torch.ones((self.batch, self.action_space_size), device=paddle_pos_new.device)
        valid[(paddle_pos_new == 0), 0] = 0
        valid[(paddle_pos_new + self.paddle_width >= self.width), -1] = 0
        return valid

    def step(self, state, action, done_mask):
        """parallel_breakout.py:158-254 through torch.ops.mz.env_step (done mutated in place and
        returned, the reference's done_mask aliasing); CPU tensors are accepted like the reference's."""
        B = self.batch
        out_dev = state.device
        s = state.to(self.device, torch.float32).contiguous()
        a = action.to(self.device, torch.int64).contiguous()
        on_dev = done_mask.device == self.device and done_mask.dtype == torch.bool and done_mask.is_contiguous()
        d = done_mask if on_dev else done_mask.to(self.device, torch.bool).contiguous()
        dx = torch.as_tensor(self.ball_dx, device=self.device).to(torch.int64).expand(B).contiguous()
        dy = torch.as_tensor(self.ball_dy, device=self.device).to(torch.float32).expand(B).contiguous()
        r4 = [float(self.paddle_hit_reward), float(self.brick_hit_reward), float(self.game_lost_reward),
              float(self.game_won_reward)]
        # a malformed state raises IndexError (TORCH_CHECK_INDEX), the reference's error type
        ns, reward, d, valid, dx, dy = L.ops().env_step(s, a, d, dx, dy, self.paddle_width, r4)
        self.ball_dx, self.ball_dy = dx, dy
        if not on_dev:
            done_mask.copy_(d)  # in place, like `done_mask |= ...` (:204, :247)
        return ns.to(out_dev), reward.to(out_dev), done_mask, valid.to(out_dev)

    def render(self, state):
        raise NotImplementedError("debug text renderer (parallel_breakout.py:257-293) is out of scope")


def grayscale(state):
    """train_torch.py:334-358 on the device: (B,3,H,W) -> (B,1,H,W)."""
    return L.ops().grayscale(state.contiguous())


GRAY_LUT = None


def gray_lut():
    """float value of each gray code (bit0 paddle, bit1 ball, bit2 brick)."""
    out = []
    for c in range(8):
        p, b, k = np.float32(c & 1), np.float32((c >> 1) & 1), np.float32((c >> 2) & 1)
        v = (p * np.float32(0.3) + b * np.float32(1.0)) + k * np.float32(0.6)
        out.append(np.clip(v, 0, 1))
    return np.array(out, dtype=np.float32)


class CompactBreakout:
    """Device-resident compact env state for B envs + frame-history ring of length L."""

    def __init__(self, cfg_env, B, L_hist, height=16, width=20, paddle_width=6, brick_rows=3, seed=0, env_offset=0,
                 device="cuda", pad_action=0, rec_flags=0, single_write=True):
        L.require_gpu()
        self.B, self.H, self.W = B, height, width
        self.pw, self.brick_rows = paddle_width, brick_rows
        self.Lh = L_hist
        self.seed, self.env_offset = seed, env_offset
        # run_test_simulation (train_torch.py:530-610): pad action 1, every env recorded with action[0]
        self.pad_action, self.rec_flags = pad_action, rec_flags
        self.rewards4 = (ctypes.c_float * 4)(cfg_env["paddle_hit_reward"], cfg_env["brick_hit_reward"],
                                             cfg_env["game_lost_reward"], cfg_env["game_won_reward"])
        dev = torch.device(device)
        self.device = dev
        i32 = lambda: torch.zeros(B, dtype=torch.int32, device=dev)  # noqa: E731
        self.paddle, self.bx, self.by, self.dx = i32(), i32(), i32(), i32()
        self.dy = torch.zeros(B, dtype=torch.float32, device=dev)
        self.done = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.nw = (brick_rows * width + 63) // 64
        self.bricks = torch.zeros(B * self.nw, dtype=torch.int64, device=dev)
        HW = height * width
        # single-write frame storage (include/mzba.h): a recorded frame lives only in the history
        # ring; cur_frame holds the live frames of done envs; cur_src[b] says which
        self.cur_frame = torch.zeros(B * HW, dtype=torch.uint8, device=dev)
        self.cur_src = torch.ones(B, dtype=torch.uint8, device=dev) if single_write else None
        self.hist_frames = torch.zeros(B * (L_hist - 1) * HW, dtype=torch.uint8, device=dev)
        self.hist_actions = torch.zeros(B * L_hist, dtype=torch.uint8, device=dev)
        self.hist_len = torch.zeros(B, dtype=torch.int32, device=dev)
        self.reward = torch.zeros(B, dtype=torch.float32, device=dev)
        self.valid = torch.ones(B, 3, dtype=torch.float32, device=dev)

    def _state_ptrs(self):
        return (L.ptr(self.paddle), L.ptr(self.bx), L.ptr(self.by), L.ptr(self.dx), L.ptr(self.dy), L.ptr(self.done),
                L.ptr(self.bricks), self.nw)

    def reset(self, episode, params=None):
        pr = None
        if params is not None:
            pr = torch.as_tensor(np.asarray(params, dtype=np.int32), device=self.device).contiguous()
        L.call("mzba_env_reset_compact", *self._state_ptrs(), L.ptr(self.cur_frame), L.ptr(self.cur_src),
               L.ptr(self.hist_frames),
               L.ptr(self.hist_actions), L.ptr(self.hist_len), self.Lh, self.B, self.H, self.W, self.pw,
               self.brick_rows, self.seed, episode, self.env_offset, L.ptr(pr), self.pad_action, L.stream())
        self.valid.fill_(1.0)

    def step(self, action, first_step, rec=None, t=0, ctx=None):
        """action: int64 (B,) device. rec: optional sink dict of (T,B,...) buffers, row t; with a
        device step context `ctx` the row (and first_step) are read on the device instead."""
        ra = rr = rm = rf = None
        if rec is not None:
            if ctx is not None:
                ra, rr, rm, rf = rec["action"], rec["reward"], rec["mask"], rec.get("frame")
            else:
                ra, rr, rm = rec["action"][t], rec["reward"][t], rec["mask"][t]
                rf = rec["frame"][t] if rec.get("frame") is not None else None
        L.call("mzba_env_step_compact", *self._state_ptrs(), L.ptr(action), L.ptr(self.reward), L.ptr(self.valid),
               L.ptr(self.cur_frame), L.ptr(self.cur_src), L.ptr(self.hist_frames), L.ptr(self.hist_actions),
               L.ptr(self.hist_len), self.Lh, L.ptr(ra), L.ptr(rr), L.ptr(rm), L.ptr(rf), 1 if first_step else 0, self.B, self.H, self.W, self.pw,
               self.brick_rows, self.rewards4, L.ptr(ctx), self.rec_flags, L.stream())

    def to_planes(self):
        planes = torch.empty(self.B, 3, self.H, self.W, dtype=torch.float32, device=self.device)
        L.call("mzba_compact_to_planes", L.ptr(self.paddle), L.ptr(self.bx), L.ptr(self.by), L.ptr(self.done),
               L.ptr(self.bricks), self.nw, L.ptr(planes), self.B, self.H, self.W, self.pw, self.brick_rows, L.stream())
        return planes

    def build_rep_input(self, out, cs, bf16):
        L.call("mzba_build_rep_input", L.ptr(self.cur_frame), L.ptr(self.cur_src), L.ptr(self.hist_frames),
               L.ptr(self.hist_actions), L.ptr(self.hist_len), self.Lh, L.ptr(out), 1 if bf16 else 0, self.B,
               self.H * self.W, cs, L.stream())

    def current_frame(self):
        """Every env's current u8 gray-code frame, (B*H*W,) on the device."""
        out = torch.empty(self.B * self.H * self.W, dtype=torch.uint8, device=self.device)
        L.call("mzba_env_current_frame", L.ptr(self.cur_frame), L.ptr(self.cur_src), L.ptr(self.hist_frames),
               L.ptr(self.hist_len), self.Lh, L.ptr(out), self.B, self.H * self.W, L.stream())
        return out
