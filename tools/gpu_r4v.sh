#!/bin/bash
# config 3 acting step kernel breakdown (rocprofv3 kernel trace, 1 timed step).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --height 84 --width 84 --hist 4 --envs 4096 --no-cpu --no-parity --steps 1 --warmup 1 > $O/prof.log 2>&1
python3 tools/rocpd_report.py stats $O/prof $O/kernel_stats_c3.csv
rm -rf $O/prof
head -25 $O/kernel_stats_c3.csv | cut -c1-200
echo r4v done
