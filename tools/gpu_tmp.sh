set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "band or nets or fused or acting" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for i in 1 2; do
for lib in libmzba_base.so libmzba.so; do
  MZBA_LIB=$PWD/muzero-breakout_amd/mzba/$lib timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu > $O/bench_${lib}_$i.json 2> $O/bench_$lib.err
  python3 -c "import json,sys; d=json.load(open('$O/bench_${lib}_$i.json')); print('$lib', round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_ms'],4))"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu > $O/prof.log 2>&1
python3 tools/rocpd_report.py stats $O/prof $O/kernel_stats_4096.csv | head -12
rm -rf $O/prof
