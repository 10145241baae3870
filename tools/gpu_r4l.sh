#!/bin/bash
# x6 with the split software-pipelined: parity tests, same-box kernel A/B against the previous commit's build,
# the headline bench with both parity paths.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
M=$PWD/muzero-breakout_amd/mzba
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "x6 or nets_f32" -x -v -s --timeout 200 --timeout-method thread \
  > $O/pytest_x6.txt 2>&1 || { tail -60 $O/pytest_x6.txt; exit 1; }
grep -E "conv_x6 |passed|failed" $O/pytest_x6.txt | tail -6
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
timeout -k 10 600 python bench.py --steps 6 --warmup 2 > $O/bench_full.json 2> $O/bench_full.err
python3 -c "import json; d=json.load(open('$O/bench_full.json')); p=d['parity_path']; print('headline', round(d['value'],1), 'match_full', d['visit_count_match_full'], 'parity x6', round(p['value'],1), 'f32mfma', round(p['vs_f32_mfma_path']['value'],1), 'x6~f32', p['vs_f32_mfma_path']['visit_count_match'], 'cpu', d['cpu_baseline']['value'])"
echo r4l done
