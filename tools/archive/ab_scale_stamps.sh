#!/bin/bash
# Same-box stamps A/B of the dynamics epilogue (towerp_kernel, fused dynamics step at B = 4096): the shipped
# stamp build (libmzba_pstamp.so) vs a variant (libmzba_pstamp_$2.so), alternated twice.
set -euo pipefail
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do
  for v in base $2; do
    lib=muzero-breakout_amd/mzba/libmzba_pstamp.so
    [ "$v" != base ] && lib=muzero-breakout_amd/mzba/libmzba_pstamp_$v.so
    MZBA_LIB=$PWD/$lib MZBA_LIB_PARTIAL=1 timeout -k 10 200 python tools/stamp_towerp.py ${MODE:-dyn} $O/st_$v.$i.json > $O/st_$v.$i.log 2>&1
    python3 -c "import json; d=json.load(open('$O/st_$v.$i.json')); print('$v', 'staging', d['staging'], d['epilogue'], d['tower_end_to_exit'], round(d['launch_wall_us'],1), round(d['clock_ghz_median'],3))"
  done
done
