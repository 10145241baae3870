"""Representation timing + output hash of ONE build of the C ABI (MZBA_LIB picks it), for same-box A/B
of two builds in alternating processes: the whole net (rep input -> scaled root latent) at the acting
batch through mzba_rep_trunk + rep_tail, HIP events, median of 20; sha256 of the latent's bytes, so two
builds that must be bit-identical can be checked on the same seeded input.
usage (GPU box): MZBA_LIB=muzero-breakout_amd/mzba/libmzba_base.so python tools/ab_lib_rep.py [B]"""
import hashlib
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
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.rand(B * 320 * 64, device="cuda", generator=g).to(torch.bfloat16)
    out = torch.empty(B * 20 * 256, dtype=torch.bfloat16, device="cuda")
    rn.use_rep_trunk = True
    rn.representation(x, out)
    torch.cuda.synchronize()
    h = hashlib.sha256(out.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]
    ms = [timed(lambda: rn.representation(x, out)) for _ in range(3)]
    print(json.dumps({"lib": os.path.basename(os.environ.get("MZBA_LIB", "libmzba.so")), "B": B,
                      "representation_ms": ms, "latent_sha": h}))


if __name__ == "__main__":
    main()
