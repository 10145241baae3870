"""Representation timing at the acting batch (default B = 4096), same box, alternating: the whole net
(rep input -> scaled root latent) with the 16x20 trunk (stem, 128-channel blocks, widening conv,
256-channel blocks) as one mzba_rep_trunk launch vs the band launches + mzba_rep_blocks; HIP events,
medians of 20.
usage (GPU box): python tools/ab_reptrunk.py [B]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ab_rep import timed, MuZeroAgent, default_config, init_state_dict, torch  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    mcfg = default_config()["model"]
    ag = MuZeroAgent(mcfg, dtype="bf16")
    ag.load_state_dict(init_state_dict(mcfg, 0))
    rn = ag.runner(B, 16, 20)
    x = torch.rand(B * 320 * 64, device="cuda").to(torch.bfloat16)
    out = torch.empty(B * 20 * 256, dtype=torch.bfloat16, device="cuda")
    res = {"B": B}
    for on in (True, False, True, False):
        rn.use_rep_trunk = on
        res.setdefault(f"representation_ms_rep_trunk_{on}", []).append(timed(lambda: rn.representation(x, out)))
    rn.use_rep_trunk = True
    # the trunk's algorithmic work per env: stem 64->128, 4 convs 128->128, widening 128->256, 6 convs 256->256
    fl = 2.0 * 320 * 9 * (64 * 128 + 4 * 128 * 128 + 128 * 256 + 6 * 256 * 256) * B
    res["trunk_gflop"] = fl / 1e9
    print(json.dumps(res))


if __name__ == "__main__":
    main()
