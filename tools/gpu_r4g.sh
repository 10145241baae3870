#!/bin/bash
# Round-4 GPU call: zero-row bank conflicts removed (halo zero block, x6 natural row + zeroing), x6 tile size by
# CU quantization and term-major MFMA issue — parity tests, the kernel A/B (tools/bench_x6.py), config 3, the
# headline with both parity paths, then SQ passes for conv_x6 / conv_halo_pipe.
# usage (repo root on the box): bash tools/gpu_r4g.sh TAG
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "x6 or nets_f32 or halo" -x -v --timeout 200 --timeout-method thread \
  > $O/pytest_x6.txt 2>&1 || { tail -60 $O/pytest_x6.txt; exit 1; }
grep -E "passed|failed" $O/pytest_x6.txt | tail -2
timeout -k 10 300 python tools/bench_x6.py > $O/bench_x6.jsonl 2> $O/bench_x6.err
cat $O/bench_x6.jsonl
timeout -k 10 400 python bench.py --height 84 --width 84 --hist 4 --envs 4096 --no-cpu --no-parity --steps 3 --warmup 1 \
  > $O/bench_c3.json 2> $O/bench_c3.err
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print('config 3', round(d['value'],1), round(r['avg_ms_per_conv'],4), round(r['frac'],4))"
timeout -k 10 600 python bench.py --steps 6 --warmup 2 > $O/bench_full.json 2> $O/bench_full.err
python3 -c "import json; d=json.load(open('$O/bench_full.json')); p=d['parity_path']; print('headline', round(d['value'],1), 'match_full', d['visit_count_match_full'], 'parity x6', round(p['value'],1), 'f32mfma', round(p['vs_f32_mfma_path']['value'],1), 'x6~f32', p['vs_f32_mfma_path']['visit_count_match'], 'cpu', d['cpu_baseline']['value'])"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-trace -d $O/ksq$i -o run -- python3 tools/bench_x6.py > $O/ksq$i.log 2>&1
  python3 tools/pmc_sq.py $O/ksq$i "conv_x6_kernel<256, 80, 1>" $O/ksq${i}_x6_80.json
  python3 tools/pmc_sq.py $O/ksq$i conv_halo_pipe_kernel $O/ksq${i}_halo_pipe.json
  rm -rf $O/ksq$i
done
echo r4g done
