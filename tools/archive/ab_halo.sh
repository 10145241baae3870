#!/bin/bash
# Same-box A/B of the halo conv (tools/bench_x6.py with HALO_ONLY=1) over C-ABI builds, alternated twice; every
# line carries an output checksum, so equal checksums across builds show bit-identical results.
# usage (repo root on the box): TAG=name LIBS="libmzba.so libmzba_variant.so" bash tools/ab_halo.sh
#   -> gpurun_out/TAG/halo_<lib>_<rep>.jsonl, commands.txt
set -euo pipefail
export TMPDIR=/tmp
: "${TAG:?TAG=...}" "${LIBS:?LIBS=\"a.so b.so\" (files under muzero-breakout_amd/mzba/)}"
O=gpurun_out/$TAG
mkdir -p $O
for i in 1 2; do
  for lib in $LIBS; do
    echo "HALO_ONLY=1 MZBA_LIB=muzero-breakout_amd/mzba/$lib python tools/bench_x6.py" >> $O/commands.txt
    HALO_ONLY=1 MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 200 python tools/bench_x6.py \
      > $O/halo_${lib%.so}_$i.jsonl 2> $O/halo_${lib%.so}_$i.err || { tail $O/halo_${lib%.so}_$i.err; exit 1; }
  done
done
