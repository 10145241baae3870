"""PMC summary of one conv kernel of a bench run (config 3's `conv_halo_kernel`): HBM bytes per launch from the
FETCH_SIZE / WRITE_SIZE passes (FETCH_SIZE x2: the gfx950 half-count of 16-B coalesced reads; both in KB) and the SQ
figures of the two SQ passes (tools/pmc_sq.py), beside the launch's algorithmic bytes, merged into a records file
that bench.py reads for the non-fused acting path (profiles/conv_counters.json).
  pmc_conv_summary.py DIR KERNEL_NAME ENVS H W OUT_JSON
DIR holds the rocprofv3 outputs fetch/, write/, sq1/, sq2/ (tools/gpu_run.sh step 'pmck')."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocpd_report import counter_values  # noqa: E402
from pmc_sq import summarize  # noqa: E402


def algorithmic_bytes(B, H, W, C=256):
    """One 3x3 C -> C conv of the latent residual blocks: input + output image (+ the residual image on the second
    conv of every block: half the launches) + the bf16 weights."""
    img = B * H * W * C * 2
    return 2 * img + 0.5 * img + 9 * C * C * 2


if __name__ == "__main__":
    d, kname, B, H, W, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
    f = counter_values(os.path.join(d, "fetch"), "FETCH_SIZE", kname)
    w = counter_values(os.path.join(d, "write"), "WRITE_SIZE", kname)
    s1 = summarize(os.path.join(d, "sq1"), kname)
    s2 = summarize(os.path.join(d, "sq2"), kname)
    fetch = float(np.mean(f)) * 1024 * 2 if f else None
    write = float(np.mean(w)) * 1024 if w else None
    rec = {"kernel_name": kname, "envs": B, "H": H, "W": W, "fetch_bytes": fetch, "write_bytes": write,
           "bytes_per_launch": fetch + write if f and w else None, "algorithmic_bytes": algorithmic_bytes(B, H, W),
           "n_samples": [len(f), len(w)], "mfma_busy": s1.get("mfma_busy"), "clock_ghz": s1.get("clock_ghz"),
           "wait_inst": s1.get("wait_inst"), "duration_ns": s1.get("duration_ns"),
           "lds_bank_conflict_frac": (s2["SQ_LDS_BANK_CONFLICT"] / s2["SQ_LDS_IDX_ACTIVE"])
           if s2.get("SQ_LDS_IDX_ACTIVE") else None,
           "source": d,
           "method": "rocprofv3 --pmc passes of their own (FETCH_SIZE; WRITE_SIZE; two SQ groups), --kernel-trace, over "
                     "the eager acting bench (--no-graph --no-cpu); traffic = mean per launch, SQ = medians"}
    db = {"records": []}
    if os.path.exists(out):
        db = json.load(open(out))
    db["records"] = [r for r in db["records"] if (r.get("envs"), r.get("H"), r.get("W"), r.get("kernel_name"))
                     != (B, H, W, kname)] + [rec]
    json.dump(db, open(out, "w"), indent=1)
    print(json.dumps(rec))
