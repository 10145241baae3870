#!/bin/bash
# SQ / GRBM counters of towerp_kernel inside the acting bench (4096 x 50, eager, 1 step): two separate
# --pmc passes (rocprofv3 does not split counters), summarized by tools/pmc_sq.py.
# usage (repo root on the box): bash tools/pmc_towerp_sq.sh TAG
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/sq1 -o run -- python3 bench.py --steps 1 --warmup 1 --no-graph --no-cpu --no-parity > $O/sq1.log 2>&1
python3 tools/pmc_sq.py $O/sq1 towerp_kernel $O/sq1.json
python3 tools/pmc_sq.py $O/sq1 rep_trunk_kernel $O/sq1_rep_trunk.json
python3 tools/pmc_sq.py $O/sq1 rep_tail_kernel $O/sq1_rep_tail.json
rm -rf $O/sq1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace -d $O/sq2 -o run -- python3 bench.py --steps 1 --warmup 1 --no-graph --no-cpu --no-parity > $O/sq2.log 2>&1
python3 tools/pmc_sq.py $O/sq2 towerp_kernel $O/sq2.json
python3 tools/pmc_sq.py $O/sq2 rep_trunk_kernel $O/sq2_rep_trunk.json
python3 tools/pmc_sq.py $O/sq2 rep_tail_kernel $O/sq2_rep_tail.json
rm -rf $O/sq2
echo sq done
