"""One acting step of the f32 parity path (bench.py's parity_path replay) on its own, for a kernel trace:
`rocprofv3 --kernel-trace --stats -- python3 tools/parity_step.py [B] [S] [X6] [HEADS] [REPS]`. Builds the f32 agent
(x6 latent convs) and an ActingLoop of B envs (default 4096) x S sims (default 50), runs consecutive eager acting
steps (the first warms scratch and code objects) and prints one JSON line per timed step. X6: the
mzba_conv_x6_set_variant to run (2 default: pixel-tiled at the 4x5 latent; 1: the round-4 pre-split form), HEADS:
mzba_heads_set_variant (1 default: f32 MFMA; 0: the FMA form); REPS timed steps (default 1). A same-box A/B
alternates processes with different X6 / HEADS."""
import json
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
from mzba.config import default_config  # noqa: E402
from mzba.weights import init_state_dict  # noqa: E402
from mzba.agent import MuZeroAgent  # noqa: E402
from mzba.acting import ActingLoop  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    x6 = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    heads = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    from mzba import _lib as L
    assert L.lib().mzba_conv_x6_set_variant(x6) == 0 and L.lib().mzba_heads_set_variant(heads) == 0
    cfg = default_config()
    cfg["num_simulations"] = S
    ag = MuZeroAgent(cfg["model"], dtype="f32")
    ag.load_state_dict(init_state_dict(cfg["model"], 0))
    loop = ActingLoop(cfg, ag, B, seed=0)
    loop.reset(0)
    ms = []
    for _ in range(1 + reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        loop.act(eager=True)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    for m in ms[1:]:
        print(json.dumps({"envs": B, "sims": S, "x6_variant": x6, "heads_variant": heads, "ms_per_step": m,
                          "env_steps_per_s": B / (m * 1e-3), "first_ms": ms[0]}), flush=True)


if __name__ == "__main__":
    main()
