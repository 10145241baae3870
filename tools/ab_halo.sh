# Same-box A/B of the halo conv (tools/bench_x6.py, HALO_ONLY) over C-ABI builds: TAG=... LIBS="a.so b.so" bash tools/ab_halo.sh
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-hr3}; mkdir -p $O
for i in 1 2; do for lib in ${LIBS:-libmzba.so libmzba_hr3.so}; do
  echo "HALO_ONLY=1 MZBA_LIB=$lib python tools/bench_x6.py" >> $O/commands.txt
  HALO_ONLY=1 MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 200 python tools/bench_x6.py > $O/halo_${lib%.so}_$i.jsonl 2> $O/halo_${lib%.so}_$i.err || { tail $O/halo_${lib%.so}_$i.err; exit 1; }
done; done
