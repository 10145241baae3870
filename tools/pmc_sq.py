"""SQ / GRBM counter summary of one rocprofv3 --pmc pass (rocpd SQLite output) for one kernel.
  pmc_sq.py DIR KERNEL_SUBSTRING [JSON_OUT]
Medians over the dispatches after the first 5 (warm-up), plus derived figures:
  clock_ghz     = GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md 'DVFS give-back')
  mfma_busy     = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
  wait_any / wait_inst / active_inst = fractions of SQ_WAVE_CYCLES"""
import json
import os
import sqlite3
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocpd_report import find_db  # noqa: E402


def summarize(d, kname):
    c = sqlite3.connect(find_db(d))
    rows = c.execute("select counter_name, value, dispatch_id from counters_collection where kernel_name like ? "
                     "order by dispatch_id", (f"%{kname}%",)).fetchall()
    names = sorted(set(r[0] for r in rows))
    out = {}
    for n in names:
        v = [r[1] for r in rows if r[0] == n]
        out[n] = statistics.median(v[5:] if len(v) > 6 else v)
    try:
        dur = c.execute("select duration from kernels where name like ?", (f"%{kname}%",)).fetchall()
        dur = [r[0] for r in dur]
        out["duration_ns"] = statistics.median(dur[5:] if len(dur) > 6 else dur)
    except sqlite3.Error:
        pass
    g = out.get("GRBM_GUI_ACTIVE")
    if g and out.get("duration_ns"):
        out["clock_ghz"] = g / 8 / out["duration_ns"]
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in out:
        out["mfma_busy"] = out["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * g / 8)
    w = out.get("SQ_WAVE_CYCLES")
    if w:
        for k, n in (("wait_any", "SQ_WAIT_ANY"), ("wait_inst", "SQ_WAIT_INST_ANY"), ("active_inst", "SQ_ACTIVE_INST_ANY")):
            if n in out:
                out[k] = out[n] / w
    return out


if __name__ == "__main__":
    res = summarize(sys.argv[1], sys.argv[2])
    print(json.dumps({"dir": sys.argv[1], **res}))
    if len(sys.argv) > 3:
        json.dump(res, open(sys.argv[3], "w"), indent=1)
