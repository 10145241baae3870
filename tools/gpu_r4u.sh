#!/bin/bash
# pre-split x6 (conv_x6p_kernel): parity tests (bit-identical to conv_x6_kernel), same-box kernel A/B, headline
# bench with both parity paths.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
M=$PWD/muzero-breakout_amd/mzba
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "x6 or nets_f32" -x -v -s --timeout 200 --timeout-method thread \
  > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
grep -E "conv_x6 |passed|failed" $O/pytest.txt | tail -6
for i in 1 2; do timeout -k 10 300 python tools/bench_x6.py >> $O/ab.jsonl 2>> $O/ab.err; done
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$O/ab.jsonl'):
    r=json.loads(l)
    if r['kernel']=='conv_x6': d[(tuple(r['shape']),r['variant'])].append(r['ms'])
for k,v in sorted(d.items(), key=str): print(k, [round(x,4) for x in v])
"
timeout -k 10 600 python bench.py --steps 6 --warmup 2 --no-cpu > $O/bench_full.json 2> $O/bench_full.err
python3 -c "import json; d=json.load(open('$O/bench_full.json')); p=d['parity_path']; print('headline', round(d['value'],1), 'match_full', d['visit_count_match_full'], 'parity x6', round(p['value'],1), 'f32mfma', round(p['vs_f32_mfma_path']['value'],1), 'x6~f32', p['vs_f32_mfma_path']['visit_count_match'])"
echo r4u done
