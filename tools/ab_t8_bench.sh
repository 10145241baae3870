#!/bin/bash
# Same-box config-2 bench A/B (1024 x 50: tower8_kernel<0, 1>) of the shipped library vs libmzba_t8sN.so
# (make t8-prod), alternated twice. usage: bash tools/ab_t8_bench.sh TAG N
set -euo pipefail
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do
  for v in base $2; do
    lib=muzero-breakout_amd/mzba/libmzba.so
    [ "$v" != base ] && lib=muzero-breakout_amd/mzba/libmzba_t8s$v.so
    MZBA_LIB=$PWD/$lib timeout -k 10 300 python bench.py --envs 1024 --no-cpu --no-parity --steps 10 --warmup 3 > $O/bench_$v.$i.json 2> $O/bench_$v.$i.err
    python3 -c "import json; d=json.load(open('$O/bench_$v.$i.json')); print('$v', round(d['value'],1), round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],4))"
  done
done
