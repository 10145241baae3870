#!/bin/bash
# Halo conv with 16-row zero blocks (single-stage and pipelined): parity tests, same-box kernel A/B against the
# previous commit's build (tools/bench_x6.py), config 3 acting with the pipelined vs the single-stage form.
set -euo pipefail
export TMPDIR=/tmp MZBA_LIB_PARTIAL=1
O=gpurun_out/$1
M=$PWD/muzero-breakout_amd/mzba
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "x6 or halo" -x -v --timeout 200 --timeout-method thread \
  > $O/pytest_halo.txt 2>&1 || { tail -60 $O/pytest_halo.txt; exit 1; }
grep -E "passed|failed" $O/pytest_halo.txt | tail -2
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
unset MZBA_LIB_PARTIAL
for v in "" "--halo-single" "" "--halo-single"; do
  timeout -k 10 400 python bench.py --height 84 --width 84 --hist 4 --envs 4096 --no-cpu --no-parity --steps 3 --warmup 1 $v \
    > $O/bench_c3.json 2> $O/bench_c3.err
  python3 -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print('config 3 $v', round(d['value'],1), round(r['avg_ms_per_conv'],4), round(r['frac'],4))" | tee -a $O/c3_ab.txt
done
echo r4i done
