#!/bin/bash
# SQ/GRBM counter passes on conv_big_bf16_kernel (tools/bench_conv_big.py driver, every shape;
# medians over its dispatches). usage: bash tools/pmc_conv_big.sh TAG
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/sq1 -o run -- python3 tools/bench_conv_big.py > $O/sq1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace -d $O/sq2 -o run -- python3 tools/bench_conv_big.py > $O/sq2.log 2>&1
python3 tools/pmc_sq.py $O/sq1 conv_big $O/sq1.json
python3 tools/pmc_sq.py $O/sq2 conv_big $O/sq2.json
rm -rf $O/sq1 $O/sq2
