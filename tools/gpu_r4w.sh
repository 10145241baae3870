#!/bin/bash
# rep_trunk: fragments zeroed on arrival (new) vs at the head of the consuming group (base); same box
set -o pipefail
mkdir -p gpurun_out/r4w
L=muzero-breakout_amd/mzba
for i in 1 2 3; do
  for lib in libmzba_base.so libmzba.so; do
    MZBA_LIB=$L/$lib timeout -k 10 120 python tools/ab_lib_rep.py >> gpurun_out/r4w/ab.jsonl || exit 1
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_repblocks.py > gpurun_out/r4w/pytest_rep.log 2>&1
