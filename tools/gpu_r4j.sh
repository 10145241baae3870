#!/bin/bash
# Halo conv wave split (8 channel slices vs pixel halves x quarters): parity tests, kernel A/B (same box), config 3.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "halo" -x -v -s --timeout 200 --timeout-method thread \
  > $O/pytest_halo.txt 2>&1 || { tail -60 $O/pytest_halo.txt; exit 1; }
grep -E "conv_halo|passed|failed" $O/pytest_halo.txt | tail -8
timeout -k 10 300 python tools/bench_x6.py > $O/ab_halo.jsonl 2> $O/ab_halo.err
grep conv_halo $O/ab_halo.jsonl
timeout -k 10 400 python bench.py --height 84 --width 84 --hist 4 --envs 4096 --no-cpu --no-parity --steps 3 --warmup 1 \
  > $O/bench_c3.json 2> $O/bench_c3.err
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print('config 3', round(d['value'],1), round(r['avg_ms_per_conv'],4), round(r['frac'],4))"
echo r4j done
