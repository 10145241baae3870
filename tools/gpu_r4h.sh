#!/bin/bash
# Same-box A/B of the conv kernels: the previous commit's build (libmzba_prev.so: shared zero row) against the
# working tree's, alternated twice (tools/bench_x6.py).
set -euo pipefail
export TMPDIR=/tmp MZBA_LIB_PARTIAL=1
O=gpurun_out/$1
M=$PWD/muzero-breakout_amd/mzba
mkdir -p $O
for i in 1 2; do
  for lib in libmzba_prev.so libmzba.so; do
    MZBA_LIB=$M/$lib timeout -k 10 300 python tools/bench_x6.py >> $O/ab_x6.jsonl 2>> $O/ab_x6.err
  done
done
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$O/ab_x6.jsonl'):
    r=json.loads(l); d[(r['kernel'],tuple(r['shape']),r['lib'],r['variant'])].append(r['ms'])
for k,v in sorted(d.items(), key=str): print(k, [round(x,4) for x in v])
"
echo r4h done
