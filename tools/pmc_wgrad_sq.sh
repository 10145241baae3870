#!/bin/bash
# SQ / GRBM counters of the learner's pixel-row weight-gradient kernel (conv_wgrad_px_kernel<1> = form 2, the
# default; <0> = form 1) under tools/bench_wgrad_segs.py: two separate --pmc passes, summarized by tools/pmc_sq.py (the median dispatch, all shapes).
# usage (repo root on the box): bash tools/pmc_wgrad_sq.sh TAG
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/sq1 -o run -- python3 tools/bench_wgrad_segs.py > $O/sq1.log 2>&1
python3 tools/pmc_sq.py $O/sq1 "conv_wgrad_px_kernel<1>" $O/sq1_form2.json
python3 tools/pmc_sq.py $O/sq1 "conv_wgrad_px_kernel<0>" $O/sq1_form1.json
rm -rf $O/sq1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace -d $O/sq2 -o run -- python3 tools/bench_wgrad_segs.py > $O/sq2.log 2>&1
python3 tools/pmc_sq.py $O/sq2 "conv_wgrad_px_kernel<1>" $O/sq2_form2.json
python3 tools/pmc_sq.py $O/sq2 "conv_wgrad_px_kernel<0>" $O/sq2_form1.json
rm -rf $O/sq2
echo sq done
