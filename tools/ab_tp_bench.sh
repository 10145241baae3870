#!/bin/bash
# Same-box headline-bench A/B of towerp k-loop schedules: the shipped library vs libmzba_scN.so builds
# (make towerp-prod SCHEDS=...), alternated twice. usage (repo root on the box): bash tools/ab_tp_bench.sh TAG "6 7"
set -euo pipefail
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do
  for v in base $2; do
    lib=muzero-breakout_amd/mzba/libmzba.so
    [ "$v" != base ] && lib=muzero-breakout_amd/mzba/libmzba_sc$v.so
    MZBA_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --no-parity --steps 8 --warmup 2 > $O/bench_$v.$i.json 2> $O/bench_$v.$i.err
    python3 -c "import json; d=json.load(open('$O/bench_$v.$i.json')); print('$v', round(d['value'],1), round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],4))"
  done
done
