#!/bin/bash
# learner: weight + bias partial sums in one launch (new) vs two (base); bit identity + same-box time, learner tests
set -o pipefail
O=gpurun_out/r4ab
mkdir -p $O
L=muzero-breakout_amd/mzba
for i in 1 2 3; do
  for lib in libmzba_base.so libmzba.so; do
    MZBA_LIB=$L/$lib timeout -k 10 180 python tools/ab_lib_learner.py bf16 >> $O/ab.jsonl || exit 1
  done
done
for lib in libmzba_base.so libmzba.so; do
  MZBA_LIB=$L/$lib timeout -k 10 180 python tools/ab_lib_learner.py f32 >> $O/ab.jsonl || exit 1
done
cat $O/ab.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learner.py > $O/pytest_learner.log 2>&1
tail -2 $O/pytest_learner.log
