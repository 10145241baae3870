"""One acting step of the f32 parity path (bench.py's parity_path replay) on its own, for a kernel trace:
`rocprofv3 --kernel-trace --stats -- python3 tools/parity_step.py [B] [S]`. Builds the f32 agent (x6 latent convs)
and an ActingLoop of B envs (default 4096) x S sims (default 50), runs two eager acting steps (the first warms
scratch and code objects) and prints the second's HIP-event time and env-steps/s as one JSON line."""
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
    cfg = default_config()
    cfg["num_simulations"] = S
    ag = MuZeroAgent(cfg["model"], dtype="f32")
    ag.load_state_dict(init_state_dict(cfg["model"], 0))
    loop = ActingLoop(cfg, ag, B, seed=0)
    loop.reset(0)
    ms = []
    for _ in range(2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        loop.act(eager=True)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    print(json.dumps({"envs": B, "sims": S, "ms_per_step": ms[-1], "env_steps_per_s": B / (ms[-1] * 1e-3),
                      "first_ms": ms[0]}))


if __name__ == "__main__":
    main()
