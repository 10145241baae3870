"""HBM traffic of the bench's dominant kernel from two rocprofv3 PMC passes over the acting bench
(eager launches): `rocprofv3 --pmc FETCH_SIZE --kernel-trace -- python3 bench.py --no-graph ...`
and the same with WRITE_SIZE (MI355X_MICROARCH.md: one counter group per pass; FETCH_SIZE x2 on
gfx950, both in KB). Every fused dynamics / prediction launch (`tower8_kernel<0, 2>` at B >= 2048,
`tower_kernel<0>` below) is one sample; the record is the mean per launch, beside the
algorithmic bytes of the same launches, merged into profiles/tower_hbm_traffic.json.

usage: pmc_tower_bench.py FETCH_DIR WRITE_DIR B KERNEL_NAME OUT_JSON [SIMS]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocpd_report import counter_values  # noqa: E402

C, HW, NB, NS = 256, 20, 14, 11


def algorithmic_bytes(B):
    """Mean algorithmic HBM bytes of one fused dynamics / prediction launch (bf16 weights and latents):
    dynamics = parent latent in + scaled latent out (current buffer + node-pool slot) + 29 3x3 convs +
    reward 1x1 conv + Linear(5120 -> 11) + act-bias table + biases + reward out; prediction = latent in +
    28 3x3 convs + policy 3x3 256->128 + value 1x1 256->128 + two Linears + biases + tree node traffic
    (one 64-B node per level walked, depth <= 5: counted as 5 nodes read + written)."""
    lat = B * HW * C * 2
    conv3 = 9 * C * C * 2
    dyn = lat + 2 * lat + (2 * NB + 1) * conv3 + C * C * 2 + NS * HW * C * 2 + HW * 3 * C * 4 + \
        (2 * NB + 2) * C * 4 + B * 4
    pred = lat + 2 * NB * conv3 + 9 * C * 128 * 2 + C * 128 * 2 + (3 + NS) * HW * 128 * 2 + \
        (2 * NB + 2) * C * 4 + B * 5 * 64 * 2
    return (dyn + pred) / 2.0


if __name__ == "__main__":
    fdir, wdir, B, kname, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4], sys.argv[5]
    f = counter_values(fdir, "FETCH_SIZE", kname)
    w = counter_values(wdir, "WRITE_SIZE", kname)
    fetch = float(np.mean(f)) * 1024 * 2 if f else None
    write = float(np.mean(w)) * 1024 if w else None
    rec = {"kernel_name": kname, "envs": B, "fetch_bytes": fetch, "write_bytes": write,
           "bytes_per_launch": fetch + write if f and w else None, "algorithmic_bytes": algorithmic_bytes(B),
           "n_samples": [len(f), len(w)],
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, --kernel-trace) over the eager acting "
                     "bench (python3 bench.py --no-graph --no-cpu), mean over every fused dynamics / prediction "
                     "launch of the dominant kernel; FETCH_SIZE x2 (gfx950 half-count of 16-B coalesced reads), KB"}
    db = {"records": []}
    if os.path.exists(out):
        db = json.load(open(out))
    db["records"] = [r for r in db["records"] if (r.get("envs"), r.get("kernel_name")) != (B, kname)] + [rec]
    json.dump(db, open(out, "w"), indent=1)
    print(json.dumps(rec))
