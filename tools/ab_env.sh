#!/bin/bash
# A/B of env step kernel builds on one box (tools/ab_env.py), interleaved, then the env GPU tests
# on the default build. usage (repo root on the box): bash tools/ab_env.sh TAG lib1 lib2 ...
set -euo pipefail
TAG=$1; shift
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for i in 1 2; do
  for lib in "$@"; do
    MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 120 python tools/ab_env.py 5 >> $O/ab_env.jsonl 2>> $O/ab_env.err
  done
done
cat $O/ab_env.jsonl
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "env or acting or episode" > $O/pytest_env.log 2>&1
tail -2 $O/pytest_env.log
