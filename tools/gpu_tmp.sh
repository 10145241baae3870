set -euo pipefail
export TMPDIR=/tmp MZBA_LIB_PARTIAL=1
O=gpurun_out/$1; mkdir -p $O
true
true
timeout -k 10 300 python tools/ab_tower_bits.py muzero-breakout_amd/mzba/libmzba_base.so muzero-breakout_amd/mzba/libmzba.so $O/bits > $O/bits.log || true
grep -c "\"bit_identical\": true" $O/bits.log || true
for i in 1 2; do
for lib in libmzba_base.so libmzba.so; do
  MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu > $O/bench_${lib}_$i.json 2> $O/bench_$lib.err
  python3 -c "import json,sys; d=json.load(open('$O/bench_${lib}_$i.json')); print('$lib', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_ms'],4))"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu > $O/prof.log 2>&1
python3 tools/rocpd_report.py stats $O/prof $O/kernel_stats_4096.csv | head -12
rm -rf $O/prof
