# A/B one box: bench_conv tower + bench.py with libmzba_old.so (previous commit, built separately) vs libmzba.so
# usage on the box: bash tools/ab_lib.sh
set -e
export TMPDIR=/tmp
O=gpurun_out/ab7
mkdir -p $O
for i in 1 2; do
  for lib in libmzba_old.so libmzba.so; do
    MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 120 python tools/bench_conv.py tower > $O/conv_${lib}_$i.log 2>&1
    MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > $O/bench_${lib}_$i.json 2>/dev/null
  done
done
