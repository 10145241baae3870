"""Env step kernel: time per step over batch sizes and frame geometries (fixed vs per-byte cost)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
from mzba.config import default_config  # noqa: E402
from mzba.env import CompactBreakout  # noqa: E402

cfg = default_config()
for (H, W, Lh) in ((84, 84, 4), (16, 20, 32)):
    for B in (64, 256, 1024, 4096, 16384):
        env = CompactBreakout(cfg["environment"], B, Lh, H, W, seed=0)
        acts = torch.randint(0, 3, (120, B), device="cuda")
        env.reset(0)
        for i in range(20):
            env.step(acts[i], i == 0)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(20, 120):
                env.step(acts[i], False)
        g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / 100
        print(f"{H}x{W} B={B}: {us:.2f} us/step (graph)  {B * (H * W + 48) / us / 1e3:.0f} GB/s", flush=True)
        del g, env
