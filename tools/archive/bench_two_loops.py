"""Acting-loop experiment: one ActingLoop of B envs vs two loops of B/2 envs (env offsets 0, B/2
— the sharding split, bit-identical per env) whose graph-replayed steps run on two streams, so one
half's small kernels (rep input, band convs, tree, env) overlap the other half's tower launches.
Prints env-steps/s for both (HIP graphs, synthetic bf16 nets)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "muzero-breakout_amd")]
import torch  # noqa: E402
from mzba.config import default_config  # noqa: E402
from mzba.weights import init_state_dict  # noqa: E402
from mzba.agent import MuZeroAgent  # noqa: E402
from mzba.acting import ActingLoop  # noqa: E402

B, S, K = int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 50, 10
cfg = default_config()
cfg["num_simulations"] = S
mcfg = cfg["model"]
agent = MuZeroAgent(mcfg, dtype="bf16", device="cuda:0")
agent.load_state_dict(init_state_dict(mcfg, 0))
res = {}
for n in (1, 2, 4, 1, 2, 4):
    mode = {1: "one", 2: "two", 4: "four"}[n]
    streams = [torch.cuda.Stream() for _ in range(n)]
    loops = []
    for i in range(n):
        with torch.cuda.stream(streams[i]):
            lp = ActingLoop(cfg, agent, B // n, seed=0, env_offset=i * (B // n))
            lp.reset(0)
            for _ in range(2):
                lp.act(eager=True)
            lp.capture()
            loops.append(lp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        for lp, st in zip(loops, streams):
            with torch.cuda.stream(st):
                lp.act()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res.setdefault(mode, []).append(B * K / dt)
    print(json.dumps({"mode": mode, "B": B, "env_steps_per_s": B * K / dt, "ms_per_step": dt / K * 1e3}), flush=True)
    del loops
    torch.cuda.synchronize()
