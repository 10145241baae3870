"""Agreement of the bf16 (and fp16-dynamics) acting step with the f32 parity path by simulation
count: one acting step of B envs from the same state / keyed randomness on each path; prints per S
the fraction of envs with identical visit counts, the count distance and the root-value difference.
usage (GPU box): python tools/parity_sweep.py [B] [S ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mzba.config import default_config  # noqa: E402
from mzba.weights import init_state_dict  # noqa: E402
from mzba.agent import MuZeroAgent  # noqa: E402
from mzba.acting import ActingLoop  # noqa: E402


def step(cfg, sd, dt, dyn, B, seed):
    ag = MuZeroAgent(cfg["model"], dtype=dt, dyn_dtype=dyn)
    ag.load_state_dict(sd)
    loop = ActingLoop(cfg, ag, B, seed=seed)
    loop.reset(0)
    loop.act(eager=True)
    torch.cuda.synchronize()
    out = {k: v[0].cpu().numpy() for k, v in loop.rec.items() if v is not None}
    del loop, ag
    torch.cuda.empty_cache()
    return out


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    sims = [int(a) for a in sys.argv[2:]] or [50, 100, 200]
    res = []
    for S in sims:
        cfg = default_config()
        cfg["num_simulations"] = S
        sd = init_state_dict(cfg["model"], 6)
        ref = step(cfg, sd, "f32", None, B, 12)
        for name, dt, dyn in (("bf16", "bf16", None), ("fp16dyn", "bf16", "fp16"), ("f32_again", "f32", None)):
            o = step(cfg, sd, dt, dyn, B, 12)
            same = (o["counts"] == ref["counts"]).all(1)
            d = np.abs(o["counts"] - ref["counts"]).sum(1)
            r = {"S": S, "B": B, "path": name, "match": float(same.mean()), "count_l1_mean": float(d.mean()),
                 "count_l1_p50": float(np.median(d)), "count_l1_max": int(d.max()),
                 "value_absdiff_mean": float(np.abs(o["values"] - ref["values"]).mean()),
                 "value_absdiff_max": float(np.abs(o["values"] - ref["values"]).max())}
            print(json.dumps(r), flush=True)
            res.append(r)
    return res


if __name__ == "__main__":
    main()
