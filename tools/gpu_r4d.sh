#!/bin/bash
# Round-4 GPU call (second part): config 3 with / without the halo conv, the full headline bench (CPU
# baseline + both parity paths), then the SQ counter passes of the product library and of
# libmzba_base.so (the per-pixel towerp write-back) on the same box.
# usage (repo root on the box): bash tools/gpu_r4d.sh TAG
set -euo pipefail
export TMPDIR=/tmp MZBA_LIB_PARTIAL=1
O=gpurun_out/$1
M=$PWD/muzero-breakout_amd/mzba
mkdir -p $O
for v in halo no-halo; do
  fl=""; [ $v = no-halo ] && fl=--no-halo
  timeout -k 10 400 python bench.py --height 84 --width 84 --hist 4 --envs 4096 --no-cpu --no-parity --steps 3 --warmup 1 $fl \
    > $O/bench_c3_$v.json 2> $O/bench_c3_$v.err
  python3 -c "import json; d=json.load(open('$O/bench_c3_$v.json')); r=d['roofline']; print('config 3 $v', round(d['value'],1), round(r['avg_ms_per_conv'],4), round(r['frac'],4), r['kernel'])"
done
timeout -k 10 600 python bench.py --steps 8 --warmup 2 > $O/bench_full.json 2> $O/bench_full.err
python3 -c "import json; d=json.load(open('$O/bench_full.json')); p=d['parity_path']; print('headline', round(d['value'],1), 'match_full', d['visit_count_match_full'], 'parity x6', round(p['value'],1), 'f32mfma', round(p['vs_f32_mfma_path']['value'],1), 'x6~f32', p['vs_f32_mfma_path']['visit_count_match'], 'cpu', d['cpu_baseline']['value'])"
bash tools/pmc_towerp_sq.sh $1/sq_new
python3 tools/sq_record.py $O/sq_new/sq1.json $O/sq_new/sq2.json 4096 towerp_kernel gpurun_out/$1/sq_new $O/tower_sq_counters.json
MZBA_LIB=$M/libmzba_base.so bash tools/pmc_towerp_sq.sh $1/sq_base
echo r4d done
