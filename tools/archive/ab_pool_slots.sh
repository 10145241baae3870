#!/bin/bash
# Same-box A/B of the search's latent path: node-pool slots directly (MZBA_POOL_SLOTS=1, default) vs
# through the contiguous `cur` buffer (0), headline bench alternated twice.
# usage (repo root on the box): bash tools/ab_pool_slots.sh TAG
set -euo pipefail
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do
  for v in 0 1; do
    MZBA_POOL_SLOTS=$v timeout -k 10 300 python bench.py --no-cpu --no-parity --steps 8 --warmup 2 > $O/bench_slots$v.$i.json 2> $O/bench_slots$v.$i.err
    python3 -c "import json; d=json.load(open('$O/bench_slots$v.$i.json')); print('slots=$v', round(d['value'],1), round(d['roofline']['avg_launch_ms'],4))"
  done
done
