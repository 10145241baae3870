#!/bin/bash
# One gpurun call: A/B of the previous library build (libmzba_base.so, built from the last commit) against
# the working tree's libmzba.so: tower bit identity, isolated tower timing, the headline bench, and one SQ /
# GRBM counter pass per library on the isolated B = 4096 tower. Any failing step ends the script.
# usage (repo root on the box): bash tools/gpu_ab.sh TAG
set -euo pipefail
export TMPDIR=/tmp MZBA_LIB_PARTIAL=1
O=gpurun_out/$1
M=$PWD/muzero-breakout_amd/mzba
mkdir -p $O
timeout -k 10 400 python tools/ab_tower_bits.py $M/libmzba_base.so $M/libmzba.so $O/bits > $O/bits.log 2>&1 || { cat $O/bits.log; exit 1; }
cat $O/bits.log
bash tools/ab_tower.sh $O/conv libmzba_base.so libmzba.so
for lib in libmzba_base.so libmzba.so; do
  MZBA_LIB=$M/$lib timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu > $O/bench_$lib.json 2> $O/bench_$lib.err
  cat $O/bench_$lib.json
done
for lib in libmzba_base.so libmzba.so; do
  export MZBA_LIB=$M/$lib
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace -d $O/sq_$lib -o run -- python3 tools/pmc_conv.py 4096 tower 14 > $O/sq_$lib.log 2>&1
done
unset MZBA_LIB
python3 tools/pmc_sq.py $O/sq_libmzba_base.so tower8 > $O/sq_summary.txt 2>&1 || true
python3 tools/pmc_sq.py $O/sq_libmzba.so tower8 >> $O/sq_summary.txt 2>&1 || true
cat $O/sq_summary.txt
echo "ab done"
