#!/bin/bash
# x6 with a 16-row zero block: parity test, same-box kernel A/B against the previous build (libmzba_prev.so).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
M=$PWD/muzero-breakout_amd/mzba
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "x6 or nets_f32" -x -q --timeout 200 --timeout-method thread \
  > $O/pytest_x6.txt 2>&1 || { tail -60 $O/pytest_x6.txt; exit 1; }
tail -1 $O/pytest_x6.txt
for i in 1 2; do
  for lib in libmzba_prev.so libmzba.so; do
    MZBA_LIB_PARTIAL=1 MZBA_LIB=$M/$lib timeout -k 10 300 python tools/bench_x6.py >> $O/ab_x6.jsonl 2>> $O/ab_x6.err
  done
done
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$O/ab_x6.jsonl'):
    r=json.loads(l)
    if r['kernel']=='conv_x6': d[(tuple(r['shape']),r['lib'])].append(r['ms'])
for k,v in sorted(d.items(), key=str): print(k, [round(x,4) for x in v])
"
echo r4n done
