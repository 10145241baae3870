#!/bin/bash
# learner (bf16, minibatch 512 x K = 5) kernel breakdown
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r4z
mkdir -p $O
timeout -k 10 300 python3 bench.py --workload learner --dtype bf16 > $O/learner_bench.json 2> $O/learner_bench.err
cat $O/learner_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --workload learner --dtype bf16 --steps 5 --warmup 2 > $O/prof.log 2>&1
python3 tools/rocpd_report.py stats $O/prof $O/kernel_stats_learner.csv
rm -rf $O/prof
head -25 $O/kernel_stats_learner.csv | cut -c1-220
