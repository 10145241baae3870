#!/bin/bash
# Round-4 GPU call: the LDS swizzle change (rep_trunk / conv_halo / conv_x6) — their parity tests, the
# headline bench, config 3, the full bench with both parity paths, then the SQ passes (towerp, rep_trunk,
# rep_tail counters).
# usage (repo root on the box): bash tools/gpu_r4e.sh TAG
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_repblocks.py tests/test_gpu_towerp.py tests/test_gpu_parity.py -k "repblocks or trunk or towerp or halo or x6 or nets_f32 or rep" -x -v --timeout 200 --timeout-method thread \
  > $O/pytest_sw.txt 2>&1 || { tail -60 $O/pytest_sw.txt; exit 1; }
tail -3 $O/pytest_sw.txt
timeout -k 10 300 python bench.py --no-cpu --no-parity --steps 8 --warmup 2 > $O/bench_head.json 2> $O/bench_head.err
python3 -c "import json; d=json.load(open('$O/bench_head.json')); r=d['roofline']; print('headline', round(d['value'],1), round(r['avg_launch_ms'],4), round(r['frac'],4))"
timeout -k 10 400 python bench.py --height 84 --width 84 --hist 4 --envs 4096 --no-cpu --no-parity --steps 3 --warmup 1 \
  > $O/bench_c3_halo.json 2> $O/bench_c3_halo.err
python3 -c "import json; d=json.load(open('$O/bench_c3_halo.json')); r=d['roofline']; print('config 3', round(d['value'],1), round(r['avg_ms_per_conv'],4), round(r['frac'],4))"
timeout -k 10 400 python bench.py --height 84 --width 84 --hist 4 --envs 4096 --no-cpu --no-parity --steps 3 --warmup 1 --halo-single \
  > $O/bench_c3_single.json 2> $O/bench_c3_single.err
python3 -c "import json; d=json.load(open('$O/bench_c3_single.json')); r=d['roofline']; print('config 3 single-stage', round(d['value'],1), round(r['avg_ms_per_conv'],4), round(r['frac'],4))"
timeout -k 10 600 python bench.py --steps 8 --warmup 2 > $O/bench_full.json 2> $O/bench_full.err
python3 -c "import json; d=json.load(open('$O/bench_full.json')); p=d['parity_path']; print('headline', round(d['value'],1), 'match_full', d['visit_count_match_full'], 'parity x6', round(p['value'],1), 'f32mfma', round(p['vs_f32_mfma_path']['value'],1), 'x6~f32', p['vs_f32_mfma_path']['visit_count_match'], 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $O/prof.log 2>&1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_full.csv \;
rm -rf $O/prof
head -25 $O/kernel_stats_full.csv | cut -c1-150
bash tools/pmc_towerp_sq.sh $1/sq
echo r4e done
