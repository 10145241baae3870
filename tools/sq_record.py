"""Merge the two SQ counter passes of tools/pmc_towerp_sq.sh (sq1.json: cycles / MFMA busy, sq2.json: MFMA
instructions / LDS) into profiles/tower_sq_counters.json, the record bench.py quotes as roofline.mfma_busy.
usage: sq_record.py SQ1_JSON SQ2_JSON ENVS KERNEL_NAME SOURCE_DIR [OUT] [SIMS] [DYN_DTYPE]
Records are keyed on (envs, kernel template instance, sims, dynamics dtype): bench.py quotes one only for the
launches it counted (config 5's fp16 dynamics step is towerp_kernel<1>)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def record(sq1, sq2, envs, kname, source, sims=50, dyn=None):
    a, b = json.load(open(sq1)), json.load(open(sq2))
    rec = {"envs": envs, "kernel_name": kname, "sims": sims, "dyn_dtype": dyn, "source": source,
           "mfma_busy": a.get("mfma_busy"), "clock_ghz": a.get("clock_ghz"), "wait_inst": a.get("wait_inst"),
           "duration_ns": a.get("duration_ns"), "sq_insts_mfma": b.get("SQ_INSTS_MFMA"),
           "executed_tflop_per_launch": b.get("SQ_INSTS_MFMA") and b["SQ_INSTS_MFMA"] * 16384 / 1e12,
           "lds_bank_conflict_frac": (b["SQ_LDS_BANK_CONFLICT"] / b["SQ_LDS_IDX_ACTIVE"]
                                      if b.get("SQ_LDS_IDX_ACTIVE") else None),
           "sq_insts_lds": b.get("SQ_INSTS_LDS")}
    return rec


if __name__ == "__main__":
    out = sys.argv[6] if len(sys.argv) > 6 else os.path.join(ROOT, "profiles", "tower_sq_counters.json")
    sims = int(sys.argv[7]) if len(sys.argv) > 7 else 50
    dyn = sys.argv[8] if len(sys.argv) > 8 and sys.argv[8] not in ("", "none", "None") else None
    rec = record(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4], sys.argv[5], sims, dyn)
    recs = json.load(open(out))["records"] if os.path.exists(out) else []
    key = lambda r: (r["envs"], r["kernel_name"], r.get("sims", 50), r.get("dyn_dtype"))  # noqa: E731
    recs = [r for r in recs if key(r) != key(rec)] + [rec]
    json.dump({"what": "SQ counters of the dominant kernel inside bench.py (rocprofv3 --pmc, two passes, "
                       "tools/gpu_run.sh sq); mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x "
                       "GRBM_GUI_ACTIVE / 8 XCDs), lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE",
               "records": recs}, open(out, "w"), indent=1)
    print(json.dumps(rec))
