# SQ / GRBM counters of the isolated B = 4096 tower on the round's last tree (MFMA busy, waits, clock)
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/sq_r2l
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace -d $O/sq -o run -- python3 tools/pmc_conv.py 4096 tower 14 > $O/sq.log 2>&1
python3 tools/pmc_sq.py $O/sq tower8 $O/sq_summary.json
echo "sq done"
