#!/bin/bash
# rep_trunk timing ablation: ring loads L2-hot (libmzba_ablw.so, results wrong) vs the product build; same box
set -o pipefail
mkdir -p gpurun_out/r4aa
L=muzero-breakout_amd/mzba
for i in 1 2 3; do
  for lib in libmzba.so libmzba_ablw.so; do
    MZBA_LIB=$L/$lib timeout -k 10 120 python tools/ab_lib_rep.py >> gpurun_out/r4aa/ab.jsonl || exit 1
  done
done
cat gpurun_out/r4aa/ab.jsonl
