"""Bit-identity A/B of two builds of the tower kernels (same seeded inputs, one process per library).

  python tools/ab_tower_bits.py LIB_A LIB_B [OUTDIR]

Each library runs, in its own subprocess (MZBA_LIB=...), the plain 14-block tower at B = 4096 / 2048 /
13 and the fused dynamics + prediction steps (random-init reference nets) at B = 4096 and 13, for
tower variants 0 (by batch) and 2 (8-env kernel); the outputs are dumped and compared bit for bit.
Prints one JSON line per case and exits non-zero on any difference."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def dump(out):
    sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
    import numpy as np
    import torch
    from mzba import _lib as L
    from mzba.agent import MuZeroAgent
    from mzba.config import default_config
    from mzba.weights import init_state_dict
    res = {}
    C = 256
    for B in (4096, 2048, 13):
        g = torch.Generator().manual_seed(B)
        nb = 14
        x = torch.rand(B * 20 * C, generator=g).to(torch.bfloat16).cuda()
        wf = (torch.randn(2 * nb * C * 2304 + 8 * 64 * 8, generator=g) * 0.02).to(torch.bfloat16).cuda()
        b = (torch.randn(2 * nb * C, generator=g) * 0.1).cuda()
        y = torch.empty_like(x)
        L.call("mzba_tower_set_variant", 2)
        L.call("mzba_tower", L.ptr(x), 20 * C, None, 0, L.ptr(y), L.ptr(wf), L.ptr(b), nb, B, None, 0, L.stream())
        L.call("mzba_tower_set_variant", 0)
        torch.cuda.synchronize()
        res[f"tower_{B}"] = y.view(torch.int16).cpu().numpy()
    mcfg = default_config()["model"]
    ag = MuZeroAgent(mcfg, dtype="bf16")
    ag.load_state_dict(init_state_dict(mcfg, 7))
    for B in (4096, 13):
        # variant 2 for the whole case: a build without mzba_tower_ext.plan picks the kernel at launch
        L.call("mzba_tower_set_variant", 2)
        rn = ag.runner(B, 16, 20)
        assert rn.fused_ok() and rn.tower_plan == 2
        S1, n = 3, 20 * 256
        g = torch.Generator().manual_seed(B)
        pool = torch.rand(B, S1 + 1, n, generator=g).to(torch.bfloat16).cuda()
        slot = torch.randint(0, S1, (B,), generator=g, dtype=torch.int32).cuda()
        act = torch.randint(0, 3, (B,), generator=g, dtype=torch.int32).cuda()
        o = torch.empty(B, n, dtype=torch.bfloat16, device="cuda")
        f = lambda *s: torch.full(s, float("nan"), device="cuda")  # noqa: E731
        r, rl, pi, v, plg, vlg = f(B), f(B, 11), f(B, 3), f(B), f(B, 3), f(B, 11)
        rn.dynamics(pool, act, o, r, rl, slot=slot, env_stride=(S1 + 1) * n, slot_stride=n, pool=pool,
                    pool_env_stride=(S1 + 1) * n, pool_slot=S1)
        torch.cuda.synchronize()
        r, rl = r.clone(), rl.clone()  # the dynamics outputs before the prediction launch runs
        rn.prediction(o, pi, v, plg, vlg)
        torch.cuda.synchronize()
        L.call("mzba_tower_set_variant", 0)
        for k, t in dict(latent=o.view(torch.int16), pool=pool[:, S1].view(torch.int16), r=r.view(torch.int32),
                         rl=rl.view(torch.int32), pi=pi.view(torch.int32), v=v.view(torch.int32),
                         plg=plg.view(torch.int32), vlg=vlg.view(torch.int32)).items():
            res[f"fused_{B}_{k}"] = t.cpu().numpy()
    np.savez(out, **res)


def main():
    import numpy as np
    a, b = sys.argv[1], sys.argv[2]
    od = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "gpurun_out", "ab_bits")
    os.makedirs(od, exist_ok=True)
    outs = []
    for i, lib in enumerate((a, b)):
        o = os.path.join(od, f"dump_{i}.npz")
        env = dict(os.environ, MZBA_LIB=os.path.abspath(lib))
        subprocess.run([sys.executable, os.path.abspath(__file__), "--dump", o], env=env, check=True, timeout=300)
        outs.append(np.load(o))
    bad = 0
    for k in outs[0].files:
        x, y = outs[0][k], outs[1][k]
        eq = bool(np.array_equal(x, y))
        bad += not eq
        print(json.dumps({"case": k, "bit_identical": eq, "n": int(x.size), "n_diff": int((x != y).sum())}))
    for i in range(2):  # the dumps are large; keep only the verdict
        os.remove(os.path.join(od, f"dump_{i}.npz"))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--dump":
        dump(sys.argv[2])
    else:
        main()
