set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 120 python tools/stamp_tower.py 4096 14 $O/stamps_4096.json
timeout -k 10 300 python tools/ab_tower_bits.py muzero-breakout_amd/mzba/libmzba_base.so muzero-breakout_amd/mzba/libmzba.so $O/bits | grep -c '"bit_identical": true'
bash tools/ab_tower.sh $O/conv libmzba_base.so libmzba.so
for lib in libmzba_base.so libmzba.so; do
  MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu > $O/bench_$lib.json 2> $O/bench_$lib.err
  python3 -c "import json,sys; d=json.load(open('$O/bench_$lib.json')); print('$lib', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_ms'],4))"
done
