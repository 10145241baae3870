"""Env render kernel sweep (config 3 geometry): envs per workgroup E -> us per step.
usage: python tools/bench_env.py [B] [H] [W] [L]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
from mzba.config import default_config  # noqa: E402
from mzba.env import CompactBreakout  # noqa: E402
from mzba import _lib as L  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
H = int(sys.argv[2]) if len(sys.argv) > 2 else 84
W = int(sys.argv[3]) if len(sys.argv) > 3 else 84
Lh = int(sys.argv[4]) if len(sys.argv) > 4 else 4
cfg = default_config()
for sw in (True, False):
    env = CompactBreakout(cfg["environment"], B, Lh, H, W, seed=0, single_write=sw)
    acts = torch.randint(0, 3, (200, B), device="cuda")
    for E in (0, 1, 2, 4, 8, 16):
        L.call("mzba_env_set_block_envs", E)
        env.reset(0)
        for i in range(20):
            env.step(acts[i], i == 0)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for i in range(20, 200):
            env.step(acts[i], False)
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / 180
        print(f"single_write={sw} E={E}: {us:.2f} us/step  {B * (H * W + 48) / us / 1e3:.0f} GB/s algorithmic", flush=True)
L.call("mzba_env_set_block_envs", 0)
