# A/B of tower builds on one box: bench_conv tower (B=1024/2048/4096, 14 blocks) per library, twice
# usage on the box: bash tools/ab_tower.sh OUTDIR lib1 lib2 ...
set -e
O=$1; shift
mkdir -p $O
for i in 1 2; do
  for lib in "$@"; do
    MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 120 python tools/bench_conv.py tower > $O/conv_${lib}_$i.log 2>&1
  done
done
for lib in "$@"; do echo "== $lib"; grep -h '"nblocks": 14' $O/conv_${lib}_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['B'], d['variant'], round(d['us'], 1), round(d['tflops'], 1))"; done
