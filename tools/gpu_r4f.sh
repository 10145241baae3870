#!/bin/bash
# Round-4 GPU call: where the time goes in config 3 (conv_halo_pipe_kernel) and in the f32 parity path
# (conv_x6_kernel): a kernel-trace profile of the headline bench with its parity replays, then SQ counter
# passes (two per workload, rocprofv3 does not split counters) of config 3 and of the headline + parity.
# usage (repo root on the box): bash tools/gpu_r4f.sh TAG
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "x6 or nets_f32 or halo" -x -v --timeout 200 --timeout-method thread \
  > $O/pytest_x6.txt 2>&1 || { tail -60 $O/pytest_x6.txt; exit 1; }
grep -E "conv_x6|passed|failed" $O/pytest_x6.txt | tail -8
for v in "" "--x6-split2"; do
  timeout -k 10 600 python bench.py --steps 4 --warmup 1 --no-cpu $v > $O/bench_par$v.json 2> $O/bench_par$v.err
  python3 -c "import json; d=json.load(open('$O/bench_par$v.json')); p=d['parity_path']; print('x6 $v', round(p['value'],1), 'f32mfma', round(p['vs_f32_mfma_path']['value'],1), 'x6~f32', p['vs_f32_mfma_path']['visit_count_match'], 'head', round(d['value'],1))"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/prof.log 2>&1
python3 tools/rocpd_report.py stats $O/prof $O/kernel_stats_full.csv
rm -rf $O/prof
head -30 $O/kernel_stats_full.csv | cut -c1-160
C3="bench.py --height 84 --width 84 --hist 4 --envs 4096 --no-cpu --no-parity --steps 1 --warmup 1 --no-graph"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-trace -d $O/c3sq$i -o run -- python3 $C3 > $O/c3sq$i.log 2>&1
  python3 tools/pmc_sq.py $O/c3sq$i conv_halo_pipe_kernel $O/c3sq${i}_halo.json
  rm -rf $O/c3sq$i
done
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-trace -d $O/psq$i -o run -- python3 bench.py --steps 1 --warmup 1 --no-graph --no-cpu > $O/psq$i.log 2>&1
  python3 tools/pmc_sq.py $O/psq$i conv_x6_kernel $O/psq${i}_x6.json
  python3 tools/pmc_sq.py $O/psq$i rep_trunk_kernel $O/psq${i}_rep_trunk.json
  python3 tools/pmc_sq.py $O/psq$i rep_tail_kernel $O/psq${i}_rep_tail.json
  rm -rf $O/psq$i
done
echo r4f done
