#!/bin/bash
# SQ/GRBM counter passes on the tower kernel (pmc_conv.py driver). usage: bash tools/pmc_tower_sq.sh TAG
set -e
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/sq1 -o run -- python3 tools/pmc_conv.py 1024 tower 14 > $O/sq1.log 2>&1 && echo sq1 ok
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace -d $O/sq2 -o run -- python3 tools/pmc_conv.py 1024 tower 14 > $O/sq2.log 2>&1 && echo sq2 ok
python3 - "$O" <<'PY'
import sys, glob, sqlite3, statistics
o = sys.argv[1]
for p in ("sq1", "sq2"):
    db = glob.glob(f"{o}/{p}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select counter_name, value, duration from counters_collection where kernel_name like '%tower_kernel%'").fetchall()
    names = sorted(set(r[0] for r in rows))
    for n in names:
        v = [r[1] for r in rows if r[0] == n][5:]
        d = [r[2] for r in rows if r[0] == n][5:]
        print(p, n, statistics.median(v), "dur_ns", statistics.median(d))
PY
