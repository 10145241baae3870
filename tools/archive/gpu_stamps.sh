#!/bin/bash
# towerp phase stamps + per-workgroup spread (dyn / pred / plain) in one gpurun call
# usage (repo root on the box): bash tools/gpu_stamps.sh TAG
set -euo pipefail
TAG=${1:-stamps}
O=gpurun_out/$TAG
mkdir -p $O
for m in dyn pred plain; do
  MZBA_LIB=$PWD/muzero-breakout_amd/mzba/libmzba_pstamp.so timeout -k 10 200 python tools/stamp_towerp.py $m $O/stamps_$m.json > $O/stamps_$m.log 2>&1
done
echo stamps done
