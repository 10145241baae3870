#!/bin/bash
# Round-4 GPU call: the GPU test suite (the new halo conv test first), then a same-box A/B of the previous
# library (libmzba_base.so) against the working tree's libmzba.so on the headline bench (alternated twice),
# the L2 weight-stream probe, config 2, config 3 with and without the halo-tiled conv, then the SQ counter
# passes of the dominant kernel. Every GPU step has its own time limit; any failure ends the script.
# usage (repo root on the box): bash tools/gpu_r4.sh TAG [skip-tests]
set -euo pipefail
export TMPDIR=/tmp MZBA_LIB_PARTIAL=1
O=gpurun_out/$1
M=$PWD/muzero-breakout_amd/mzba
mkdir -p $O
if [ "${2:-}" != skip-tests ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "halo or x6 or nets_f32" -x -v -s --timeout 200 --timeout-method thread \
    > $O/pytest_halo.txt 2>&1 || { tail -60 $O/pytest_halo.txt; exit 1; }
  grep -E "conv_halo|conv_x6|passed|failed" $O/pytest_halo.txt | tail -12
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
    > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
  tail -3 $O/pytest.txt
fi
for i in 1 2; do
  for lib in libmzba_base.so libmzba.so; do
    MZBA_LIB=$M/$lib timeout -k 10 300 python bench.py --no-cpu --no-parity --steps 8 --warmup 2 > $O/bench_${lib}_$i.json 2> $O/bench_${lib}_$i.err
    python3 -c "import json; d=json.load(open('$O/bench_${lib}_$i.json')); r=d['roofline']; print('$lib', round(d['value'],1), round(r['avg_launch_ms'],4), round(r['frac'],4))"
  done
done
timeout -k 10 120 tools/probes/l2_stream_probe > $O/l2_stream.jsonl 2> $O/l2_stream.err
cat $O/l2_stream.jsonl
timeout -k 10 300 python bench.py --envs 1024 --no-cpu --no-parity --steps 8 --warmup 2 > $O/bench_1024.json 2> $O/bench_1024.err
python3 -c "import json; d=json.load(open('$O/bench_1024.json')); r=d['roofline']; print('config 2', round(d['value'],1), round(r['avg_launch_ms'],4), round(r['frac'],4))"
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
echo r4 done
