#!/bin/bash
# Same-box A/B of towerp k-loop schedules (stamp builds: libmzba_pstamp.so = TP_SCHED 1, the shipped one;
# libmzba_pstamp_scN.so), the isolated 14-block tower at B = 4096, alternated twice.
# usage (repo root on the box): bash tools/ab_tp_sched.sh TAG "5 6"
set -euo pipefail
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do
  for v in base $2; do
    lib=muzero-breakout_amd/mzba/libmzba_pstamp.so
    [ "$v" != base ] && lib=muzero-breakout_amd/mzba/libmzba_pstamp_sc$v.so
    MZBA_LIB=$PWD/$lib MZBA_LIB_PARTIAL=1 timeout -k 10 200 python tools/stamp_towerp.py plain $O/st_$v.$i.json > $O/st_$v.$i.log 2>&1
    python3 -c "import json; d=json.load(open('$O/st_$v.$i.json')); print('$v', d['per_conv_median_cycles'], round(d['launch_wall_us'],1), round(d['clock_ghz_median'],3))"
  done
done
