#!/bin/bash
# Same-box A/B of bench.py over C-ABI builds: every library in LIBS runs the same bench arguments, alternated
# REPS times (a drifting box clock shows in every build). MZBA_LIB switches the kernels under the torch ops too
# (every build carries the soname libmzba.so, csrc/Makefile).
# usage (repo root on the box): bash tools/ab_bench.sh TAG REPS "LIB1 LIB2 ..." BENCH_ARGS...
#   LIBn: file names under muzero-breakout_amd/mzba/   -> gpurun_out/TAG/<lib>_<rep>.json, commands.txt
set -euo pipefail
TAG=$1
REPS=$2
LIBS=$3
shift 3
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for i in $(seq 1 $REPS); do
  for lib in $LIBS; do
    echo "MZBA_LIB=muzero-breakout_amd/mzba/$lib python bench.py $* > $O/${lib%.so}_$i.json" >> $O/commands.txt
    MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 300 python bench.py "$@" > $O/${lib%.so}_$i.json 2> $O/${lib%.so}_$i.err \
      || { tail -20 $O/${lib%.so}_$i.err; exit 1; }
    echo "$lib rep $i: $(python3 tools/bench_summary.py $O/${lib%.so}_$i.json)"
  done
done
