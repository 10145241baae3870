#!/bin/bash
# A/B of conv_big_bf16_kernel builds on one box (tools/bench_conv_big.py), interleaved, then the
# large-conv GPU parity tests on the default build. usage: bash tools/ab_conv_big.sh TAG lib1 lib2 ...
set -euo pipefail
TAG=$1; shift
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for i in 1 2; do
  for lib in "$@"; do
    echo "== $lib $i" >> $O/ab.log
    MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 120 python tools/bench_conv_big.py >> $O/ab.log 2>> $O/ab.err
  done
done
cat $O/ab.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv_big or 84x84" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
