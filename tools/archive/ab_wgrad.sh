# A/B one box: wgrad kernel microbench + learner bench, libmzba_old.so (previous commit) vs libmzba.so
# usage on the box: bash tools/ab_wgrad.sh <outdir>
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-abw}
mkdir -p $O
for i in 1 2; do
  for lib in libmzba_old.so libmzba.so; do
    MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 120 python tools/bench_wgrad_segs.py > $O/wseg_${lib}_$i.log 2>&1
    MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 200 python bench.py --workload learner --steps 20 --warmup 5 --no-cpu > $O/learner_${lib}_$i.json 2>/dev/null
  done
done
