"""Env step kernel A/B: graph-replayed env steps (as bench.py --workload env times them), one JSON
line per geometry: us per launch incl. inter-launch gaps and algorithmic GB/s. The library is the
one MZBA_LIB names (tools/ab_env.sh runs several builds on one box).
usage: python tools/ab_env.py [reps]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
from mzba.config import default_config  # noqa: E402
from mzba.env import CompactBreakout  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfg = default_config()
lib = os.path.basename(os.environ.get("MZBA_LIB", "libmzba.so"))
for (H, W, Lh, B) in ((84, 84, 4, 4096), (84, 84, 4, 16384), (16, 20, 32, 4096), (16, 20, 32, 64)):
    env = CompactBreakout(cfg["environment"], B, Lh, H, W, seed=0)
    n = 100
    acts = torch.randint(0, 3, (n + 20, B), device="cuda")
    env.reset(0)
    for i in range(20):
        env.step(acts[i], i == 0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for i in range(20, 20 + n):
                env.step(acts[i], False)
        g.replay()
    torch.cuda.synchronize()
    best = []
    for r in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            a.record(s)
            g.replay()
            b.record(s)
        torch.cuda.synchronize()
        best.append(a.elapsed_time(b) * 1e3 / n)
    us = min(best)
    print(json.dumps({"lib": lib, "H": H, "W": W, "L": Lh, "B": B, "us_per_step": us, "us_all": best,
                      "GBps_algorithmic": B * (H * W + 48) / us / 1e3}), flush=True)
    del g, env
