#!/bin/bash
# TCP/TA counter pass on the tower kernel for the default build and ablations 1 and 3.
# usage: bash tools/pmc_tower_tcp.sh TAG
set -e
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for v in def ab3 ab4; do
  if [ $v = def ]; then unset MZBA_LIB; else export MZBA_LIB=muzero-breakout_amd/mzba/libmzba_$v.so; fi
  timeout -k 10 200 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_BUSY_avr GRBM_GUI_ACTIVE --kernel-trace -d $O/$v -o run -- python3 tools/pmc_conv.py 1024 tower 14 > $O/$v.log 2>&1 && echo $v ok
  timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_BUSY_avr TD_TD_BUSY_avr --kernel-trace -d $O/${v}_b -o run -- python3 tools/pmc_conv.py 1024 tower 14 > $O/${v}_b.log 2>&1 && echo $v b ok
done
python3 - "$O" <<'PY'
import sys, glob, sqlite3, statistics
o = sys.argv[1]
for p in ("def", "ab3", "ab4", "def_b", "ab3_b", "ab4_b"):
    dbs = glob.glob(f"{o}/{p}/**/*.db", recursive=True)
    if not dbs:
        print(p, "no db"); continue
    c = sqlite3.connect(dbs[0])
    rows = c.execute("select counter_name, value, duration from counters_collection where kernel_name like '%tower_kernel%'").fetchall()
    for n in sorted(set(r[0] for r in rows)):
        v = [r[1] for r in rows if r[0] == n][5:]
        d = [r[2] for r in rows if r[0] == n][5:]
        print(p, n, statistics.median(v), "dur_ns", statistics.median(d))
PY
